# round 4 PMC passes for the committed traffic / limiter records: C2 wf_bounce_rr, perf-1M wf_trace_pt2 (one pool)
set -o pipefail
mkdir -p gpurun_out
PMC_PASSES="1 4 5 6 7" bash scripts/pmc_valu.sh r4c2 --config c2 --steps 2 --warmup 0 --strong-spp 0 --no-extras || exit 99
PMC_PASSES="1 4 5 6 7" bash scripts/pmc_valu.sh r4bumpy --config bumpy1m --steps 2 --warmup 0 --strong-spp 0 --no-extras || exit 99
python3 scripts/pmc_traffic.py gpurun_out/pmcv_r4c2 c2_1024x1024_r16_ordered_wavefront/bounce "wf_bounce_rr<true, false, false>"
python3 scripts/pmc_traffic.py gpurun_out/pmcv_r4bumpy bumpy1m_1024x1024_r16_ordered_wavefront/trace "wf_trace_pt2"

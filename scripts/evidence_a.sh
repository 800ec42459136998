#!/usr/bin/env bash
# First half of scripts/evidence.sh (smoke, GPU suite, PMC passes recorded with the library's build id), for calls
# that must stay short.   usage: scripts/evidence_a.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -30 gpurun_out/pytest_$tag.log; exit 98; }
tail -1 gpurun_out/pytest_$tag.log
S="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
T="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for cfg in c2 bumpy1m c5 c3; do
  scripts/pmc_groups.sh ${tag}_$cfg "FETCH_SIZE" "WRITE_SIZE" "$S" "$T" -- --config $cfg --strong-spp 0 --no-extras > /dev/null || exit 99
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c2 c2_1024x1024_r16_ordered_wavefront/bounce "wf_bounce_rr<true, false, false, false, false>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_bumpy1m bumpy1m_1024x1024_r16_ordered_wavefront/trace "wf_trace_pt2<true, false, 4>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c5 c5_4096x4096_r16_ordered_wavefront/extend "wf_trace_pt<64, true, false, false, 4>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c5 c5_4096x4096_r16_ordered_wavefront/shadow "wf_trace_pt<64, true, true, false, 4>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c3 c3_1024x1024_r16_ordered_wavefront/trace "wf_trace_pt2<true, false, 4>" || exit 97
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$tag.json
cat gpurun_out/smoke_$tag.log

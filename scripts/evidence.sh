#!/usr/bin/env bash
# Round evidence on the final build: smoke, GPU suite, bench lines of every configuration, a kernel trace + stats of
# the default bench command, and the PMC passes (HBM bytes, VALU / wait counters, L2) of the dominant kernels of C2,
# perf-1M and C5, recorded with the library's build id (scripts/pmc_traffic.py) so bench.py's `traffic` / `limiter`
# come from the instantiation the line times.   usage: scripts/evidence.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -30 gpurun_out/pytest_$tag.log; exit 98; }
tail -1 gpurun_out/pytest_$tag.log
# PMC passes first (the bench lines below then carry traffic / limiter of this build)
S="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
T="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for cfg in c2 bumpy1m c5; do
  scripts/pmc_groups.sh ${tag}_$cfg "FETCH_SIZE" "WRITE_SIZE" "$S" "$T" -- --config $cfg --strong-spp 0 --no-extras > /dev/null || exit 99
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c2 c2_1024x1024_r16_ordered_wavefront/bounce "wf_bounce_rr<true, false, false, false, false>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_bumpy1m bumpy1m_1024x1024_r16_ordered_wavefront/trace "wf_trace_pt2<true, false>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c5 c5_4096x4096_r16_ordered_wavefront/extend "wf_trace_pt<64, true, false, false, true>" || exit 97
python3 scripts/pmc_traffic.py gpurun_out/pmc_${tag}_c5 c5_4096x4096_r16_ordered_wavefront/shadow "wf_trace_pt<64, true, true, false, true>" || exit 97
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$tag.json
scripts/gpu_step.sh 500 gpurun_out/bench_$tag.log python bench.py || exit 99
for cfg in c1 c3 c4 c5 bumpy1m; do
  scripts/gpu_step.sh 400 gpurun_out/bench_${tag}_$cfg.log python bench.py --config $cfg --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 || exit 99
done
grep -h "^{" gpurun_out/bench_$tag.log gpurun_out/bench_${tag}_*.log > gpurun_out/bench_lines_$tag.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
cat gpurun_out/smoke_$tag.log
python3 -c "
import json
for l in open('gpurun_out/bench_lines_$tag.jsonl'):
    d = json.loads(l); r = d.get('roofline') or {}
    print(d['config']['config'], d['value'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'limiter', bool(r.get('limiter')))"

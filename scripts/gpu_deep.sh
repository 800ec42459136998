#!/usr/bin/env bash
# deep-BVH traversal iteration: wide parity tests, bumpy1m bench, per-dispatch kernel trace
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 300 gpurun_out/pytest_wide.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or persistent or variants" || exit 99
grep -q " passed" gpurun_out/pytest_wide.log && ! grep -q "failed" gpurun_out/pytest_wide.log || { tail -40 gpurun_out/pytest_wide.log; exit 98; }
scripts/gpu_step.sh 300 gpurun_out/bench_bumpy1m.log python bench.py --config bumpy1m --steps 4 --no-cpu || exit 99
scripts/prof_trace.sh bumpy1m --config bumpy1m --steps 1 --warmup 0 || exit 99
db=$(ls gpurun_out/prof_bumpy1m/*/*.db gpurun_out/prof_bumpy1m/*.db 2>/dev/null | head -1)
python3 scripts/rocpd_summary.py "$db" wf_ > gpurun_out/prof_bumpy1m/summary.txt
tail -1 gpurun_out/pytest_wide.log
python3 -c "
import json
l=json.loads(open('gpurun_out/bench_bumpy1m.log').readline()); r=l['roofline']
print(l['value'], r['kernel'], r['frac'], r['avg_launch_ms'], r['nodes_per_query'], r['prims_per_query'], r['stage_ms'])"
head -12 gpurun_out/prof_bumpy1m/summary.txt

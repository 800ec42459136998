#!/usr/bin/env bash
# GPU parity tests, then A/B of the 4-wide traversal on the deep-BVH configurations
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || { tail -40 gpurun_out/pytest_gpu.log; exit 98; }
for cfg in c3 bumpy1m; do
  scripts/gpu_step.sh 300 gpurun_out/bench_${cfg}_wide.log python bench.py --config $cfg --steps 4 --no-cpu || exit 99
  NH_WIDE=0 scripts/gpu_step.sh 300 gpurun_out/bench_${cfg}_bin.log python bench.py --config $cfg --steps 4 --no-cpu || exit 99
done
tail -1 gpurun_out/pytest_gpu.log
for f in gpurun_out/bench_*_wide.log gpurun_out/bench_*_bin.log; do echo "== $f"; python3 -c "
import json,sys
l=json.loads(open('$f').readline())
r=l['roofline']
print(l['value'], r['kernel'], r['frac'], r['avg_launch_ms'], r['nodes_per_query'], r['prims_per_query'], r['stage_ms'])
"; done

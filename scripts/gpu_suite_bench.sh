#!/usr/bin/env bash
# GPU suite + default bench line (+ optional extra bench args as one quoted string per config)
# usage: scripts/gpu_suite_bench.sh TAG ["bench args"]...
set -u
tag=$1; shift
mkdir -p gpurun_out
scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -40 gpurun_out/pytest_$tag.log; exit 98; }
tail -1 gpurun_out/pytest_$tag.log
scripts/gpu_step.sh 400 gpurun_out/bench_$tag.log python bench.py || exit 99
tail -c 600 gpurun_out/bench_$tag.log
i=0
for a in "$@"; do
  i=$((i+1))
  scripts/gpu_step.sh 400 gpurun_out/bench_${tag}_$i.log python bench.py $a || exit 99
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/bench_${tag}_$i.log') if x.startswith('{')][0]; l=json.loads(l); r=l['roofline'] or {}
print('$a ->', l['value'], l['ms_per_step'], r.get('kernel'), r.get('frac'), r.get('avg_launch_ms'))"
done

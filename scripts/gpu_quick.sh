#!/usr/bin/env bash
# Quick GPU iteration: a pytest -k selection of the GPU parity tests, then bench lines for configs.
# usage: scripts/gpu_quick.sh "<pytest -k expr or ALL>" cfg[:steps] ...
set -u
mkdir -p gpurun_out
sel=$1; shift
if [ "$sel" = ALL ]; then karg=(); else karg=(-k "$sel"); fi
scripts/gpu_step.sh 400 gpurun_out/pytest_quick.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${karg[@]}" || exit 99
grep -q " passed" gpurun_out/pytest_quick.log && ! grep -q "failed\|error" gpurun_out/pytest_quick.log || { tail -40 gpurun_out/pytest_quick.log; exit 98; }
tail -2 gpurun_out/pytest_quick.log | head -1
for spec in "$@"; do
  cfg=${spec%%:*}; steps=${spec#*:}; [ "$steps" = "$spec" ] && steps=4
  scripts/gpu_step.sh 300 gpurun_out/bench_q_$cfg.log python bench.py --config $cfg --no-cpu --steps $steps || exit 99
  python3 -c "
import json
l=json.loads(open('gpurun_out/bench_q_$cfg.log').readline()); r=l['roofline']
print('$cfg', l['value'], r['kernel'], r['frac'], r['avg_launch_ms'], r['stage_ms'])"
done

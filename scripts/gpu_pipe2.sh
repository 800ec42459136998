#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 300 gpurun_out/pytest_pipe.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipelined or wide or variants" || exit 99
grep -q " passed" gpurun_out/pytest_pipe.log && ! grep -q "failed" gpurun_out/pytest_pipe.log || { tail -40 gpurun_out/pytest_pipe.log; exit 98; }
tail -1 gpurun_out/pytest_pipe.log
for cfg in c2 bumpy1m c3; do
  scripts/gpu_step.sh 300 gpurun_out/bench_$cfg.log python bench.py --config $cfg --no-cpu --steps $([ $cfg = c2 ] && echo 16 || echo 4) || exit 99
  python3 -c "
import json
l=json.loads(open('gpurun_out/bench_$cfg.log').readline()); r=l['roofline']
print('$cfg', l['value'], r['kernel'], r['frac'], r['avg_launch_ms'], r['stage_ms'], r['timed'])"
done
scripts/gpu_step.sh 400 gpurun_out/bench_c5.log python bench.py --config c5 --no-cpu --steps 1 --warmup 0 || exit 99
python3 -c "
import json
l=json.loads(open('gpurun_out/bench_c5.log').readline()); r=l['roofline']
print('c5', l['value'], r['kernel'], r['frac'], r['avg_launch_ms'], r['stage_ms'])"

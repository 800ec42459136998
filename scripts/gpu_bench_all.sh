#!/usr/bin/env bash
# parity tests, then the benchmark configurations, each step time-limited
set -u
scripts/gpu_step.sh 400 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 99
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 98; }
scripts/gpu_step.sh 300 gpurun_out/bench_c2.log python bench.py || exit 99
scripts/gpu_step.sh 300 gpurun_out/bench_c1.log python bench.py --config c1 --no-cpu || exit 99
scripts/gpu_step.sh 400 gpurun_out/bench_bumpy1m.log python bench.py --config bumpy1m --steps 4 --no-cpu || exit 99
tail -1 gpurun_out/pytest_gpu.log
for f in c2 c1 bumpy1m; do echo "== $f"; head -c 1500 gpurun_out/bench_$f.log; echo; done

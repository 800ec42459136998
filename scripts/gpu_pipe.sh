#!/usr/bin/env bash
# full GPU parity suite, then pooled vs single-pool A/B on C2 and bumpy1m
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || { tail -40 gpurun_out/pytest_gpu.log; exit 98; }
tail -1 gpurun_out/pytest_gpu.log
scripts/sweep_env.sh NH_POOLS "2 1" --config c2 --no-cpu || exit 99
scripts/sweep_env.sh NH_POOLS "2 1" --config bumpy1m --steps 4 --no-cpu || exit 99

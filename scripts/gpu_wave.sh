#!/usr/bin/env bash
# parity tests (both modes), then megakernel vs wavefront benches on c2 and bumpy1m
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x -rA || exit 99
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || { tail -40 gpurun_out/pytest_gpu.log; exit 98; }
scripts/gpu_step.sh 300 gpurun_out/bench_c2_wave.log python bench.py --mode wavefront --no-cpu || exit 99
scripts/gpu_step.sh 400 gpurun_out/bench_bumpy1m_wave.log python bench.py --config bumpy1m --steps 4 --no-cpu --mode wavefront || exit 99
scripts/gpu_step.sh 400 gpurun_out/bench_bumpy1m_mega.log python bench.py --config bumpy1m --steps 4 --no-cpu || exit 99
tail -3 gpurun_out/pytest_gpu.log
for f in c2_wave bumpy1m_wave bumpy1m_mega; do echo "== $f"; tail -c 1800 gpurun_out/bench_$f.log; echo; done

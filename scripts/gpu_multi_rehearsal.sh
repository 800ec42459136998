#!/usr/bin/env bash
# 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo framebuffer reduce), then C5 and C4 lines.
set -u
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
scripts/gpu_step.sh 400 gpurun_out/bench_gloo2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --no-cpu || exit 99
tail -2 gpurun_out/bench_gloo2.log
scripts/gpu_step.sh 400 gpurun_out/bench_c5.log python bench.py --config c5 --no-cpu --steps 1 --warmup 1 || exit 99
head -1 gpurun_out/bench_c5.log | cut -c1-400
scripts/gpu_step.sh 400 gpurun_out/bench_c4.log python bench.py --config c4 --no-cpu --steps 2 || exit 99
head -1 gpurun_out/bench_c4.log | cut -c1-400

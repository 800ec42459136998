#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
scripts/prof_trace.sh c2 --config c2 --steps 2 --warmup 1 || exit 99
db=$(ls gpurun_out/prof_c2/*/*.db gpurun_out/prof_c2/*.db 2>/dev/null | head -1)
python3 scripts/rocpd_summary.py "$db" "" > gpurun_out/prof_c2/summary.txt
head -12 gpurun_out/prof_c2/summary.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --dist-backend gloo --no-cpu > gpurun_out/bench_gloo2.log 2>&1 || { tail -20 gpurun_out/bench_gloo2.log; exit 99; }
grep "^{" gpurun_out/bench_gloo2.log | cut -c1-600

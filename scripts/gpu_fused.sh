#!/usr/bin/env bash
# fused splat + async tails: parity tests, A/B on C2 / C4 / C1, then the whole GPU suite
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_splat or async_tails" -x -v --timeout 250 --timeout-method thread > gpurun_out/t_fused.log 2>&1 || { tail -30 gpurun_out/t_fused.log; exit 99; }
tail -2 gpurun_out/t_fused.log
scripts/ab_env.sh 1 "c2 c4" "NH_SPLAT_FUSED=0 NH_SPLAT_FUSED=1" --steps 8 --warmup 2 > gpurun_out/ab_fused.txt 2>&1 || { cat gpurun_out/ab_fused.txt; exit 99; }
cat gpurun_out/ab_fused.txt
scripts/ab_env.sh 1 "c1 c4" "NH_TAIL_ASYNC=0 NH_TAIL_ASYNC=1" --steps 8 --warmup 2 > gpurun_out/ab_tail.txt 2>&1 || { cat gpurun_out/ab_tail.txt; exit 99; }
cat gpurun_out/ab_tail.txt
scripts/gpu_quick.sh ALL > gpurun_out/quick_all.txt 2>&1 || { tail -30 gpurun_out/quick_all.txt; exit 99; }
tail -3 gpurun_out/quick_all.txt

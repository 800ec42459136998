#!/usr/bin/env bash
# async tails x tail workgroup size on the specular configs
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_splat or async_tails or variants or pipelined" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_tail.log 2>&1 || { tail -30 gpurun_out/t_tail.log; exit 99; }
tail -1 gpurun_out/t_tail.log
scripts/ab_env.sh 1 "c1 c4" "NH_TAIL_ASYNC=0,NH_TAIL_WG=256 NH_TAIL_ASYNC=0,NH_TAIL_WG=64 NH_TAIL_ASYNC=1,NH_TAIL_WG=64" --steps 8 --warmup 2 || exit 99

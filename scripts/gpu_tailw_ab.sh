#!/usr/bin/env bash
# tail register budget (NH_TAIL_RR_WAVES 1: ~250 VGPRs, 4: 128 VGPRs with spills) on C1 / C4 / C2
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "async_tails or variants or pipelined or parity_cbox" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_tailw.log 2>&1 || { tail -30 gpurun_out/t_tailw.log; exit 99; }
tail -1 gpurun_out/t_tailw.log
scripts/ab_env.sh 2 "c1 c4 c2" "NH_TAIL_RR_WAVES=1 NH_TAIL_RR_WAVES=4" --steps 8 --warmup 2 || exit 99

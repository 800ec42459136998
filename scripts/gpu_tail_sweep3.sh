#!/usr/bin/env bash
# fused-bounce tail threshold with the round-3 tail kernel (64-thread, 128-VGPR workgroups); default 65536 at C2/C4 sizes
set -u
mkdir -p gpurun_out
scripts/ab_env.sh 2 "c2 c4 c1" "NH_TAIL=65536 NH_TAIL=131072 NH_TAIL=262144 NH_TAIL=32768" --steps 8 --warmup 2 || exit 99

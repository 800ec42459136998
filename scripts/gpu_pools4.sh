#!/usr/bin/env bash
# pools in flight on the specular configs with the cheaper tails (64-thread, 128-VGPR tail workgroups)
set -u
mkdir -p gpurun_out
scripts/ab_env.sh 2 "c1 c4" "NH_POOLS=3 NH_POOLS=4" --steps 8 --warmup 2 || exit 99

#!/usr/bin/env bash
# wf_bounce_rr register budget: 4 waves/SIMD (default build) vs 3 (lib_w3: -DNH_BOUNCE_WAVES=3)
set -u
mkdir -p gpurun_out
for c in c2 c4; do echo "== $c"; scripts/ab_libs.sh 2 "lib lib_w3" --config $c --steps 8 --warmup 2 || exit 99; done

#!/usr/bin/env bash
# closing evidence (smoke, GPU suite, default bench, rocprofv3 trace, C1/C4/C3/C5) then the pools A/B
set -u
scripts/round3_evidence.sh r3c || exit 99
scripts/ab_env.sh 2 "c1 c4" "NH_POOLS=3 NH_POOLS=4" --steps 8 --warmup 2 > gpurun_out/pools34.txt 2>&1 || exit 99
cat gpurun_out/pools34.txt

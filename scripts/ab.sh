#!/usr/bin/env bash
# A/B of two library builds in one GPU session: scripts/ab.sh ROUNDS bench-args...
# A = optix-renderer_amd/lib (current), B = optix-renderer_amd/lib_alt; interleaved runs.
set -u
n=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in A B; do
    if [ $v = B ]; then export NH_LIB_PATH=$PWD/optix-renderer_amd/lib_alt/libnori_hip.so; else unset NH_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu --no-calibrate "$@" > gpurun_out/ab_$v$i.log 2>&1 || { echo "fail $v$i"; tail -3 gpurun_out/ab_$v$i.log; exit 99; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab_$v$i.log').read().strip().splitlines()[-1])
print('$v$i', d['value'], d['ms_per_step'])"
  done
done

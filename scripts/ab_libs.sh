#!/usr/bin/env bash
# Interleaved A/B of library builds: scripts/ab_libs.sh ROUNDS "lib lib_w5 ..." bench-args...
set -u
n=$1; libs=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in $libs; do
    if [ $v = lib ]; then unset NH_LIB_PATH; else export NH_LIB_PATH=$PWD/optix-renderer_amd/$v/libnori_hip.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 "$@" > gpurun_out/abl_$v$i.log 2>&1 || { echo "fail $v$i"; tail -3 gpurun_out/abl_$v$i.log; exit 99; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/abl_$v$i.log').read().strip().splitlines()[-1])
print('$v$i', d['value'], d['ms_per_step'])"
  done
done

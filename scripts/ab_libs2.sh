#!/usr/bin/env bash
# Interleaved A/B of library builds with the roofline pass (splat and dominant-kernel launch times):
# scripts/ab_libs2.sh ROUNDS "lib lib_v1 ..." bench-args...
set -u
n=$1; libs=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in $libs; do
    if [ $v = lib ]; then unset NH_LIB_PATH; else export NH_LIB_PATH=$PWD/optix-renderer_amd/$v/libnori_hip.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-denoise --traversal-1m-steps 0 "$@" > gpurun_out/abl2_$v$i.log 2>&1 || { echo "fail $v$i"; tail -3 gpurun_out/abl2_$v$i.log; exit 99; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/abl2_$v$i.log') if x.startswith('{')][0]); r=d['roofline'] or {}
print('$v$i', d['value'], d['ms_per_step'], 'splat', r.get('splat_ms_per_launch'), r.get('kernel','')[:14], r.get('avg_launch_ms'))"
  done
done

#!/usr/bin/env bash
# perf-1M traversal A/B: lib vs lib_alt, bench's traversal_1m record (kernel frac) + bumpy-1M / C3 lines
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for v in lib lib_alt; do
    if [ $v = lib ]; then unset NH_LIB_PATH; else export NH_LIB_PATH=$PWD/optix-renderer_amd/$v/libnori_hip.so; fi
    timeout -k 10 300 python bench.py --config bumpy1m --steps 4 --no-cpu --no-denoise > gpurun_out/abt_$v$i.log 2>&1 || { echo "fail $v$i"; tail -3 gpurun_out/abt_$v$i.log; exit 99; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abt_$v$i.log') if l.startswith('{')][-1])
r=d['roofline']
print('$v$i bumpy1m', d['value'], d['ms_per_step'], r['kernel'][:12], r['frac'], r['avg_launch_ms'])"
  done
done

#!/usr/bin/env bash
# tail threshold on C2 / bumpy-1M / C4 + fused-bounce occupancy variants on C2
set -u
mkdir -p gpurun_out
run() {  # tag env... -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 "$@" > gpurun_out/sw_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/sw_$tag.log; exit 99; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/sw_$tag.log').read().strip().splitlines()[-1])
print('$tag', d['value'], d['ms_per_step'])"
}
W5=NH_LIB_PATH=$PWD/optix-renderer_amd/lib_w5/libnori_hip.so
W3=NH_LIB_PATH=$PWD/optix-renderer_amd/lib_w3/libnori_hip.so
for i in 1 2; do
  run c2def$i X=1 -- --steps 16
  run c2t64k$i NH_TAIL=65536 -- --steps 16
  run c2w5$i $W5 -- --steps 16
  run c2w3$i $W3 -- --steps 16
  run c4t32k$i NH_TAIL=32768 -- --config c4 --steps 8
  run c4t64k$i NH_TAIL=65536 -- --config c4 --steps 8
  run b1mdef$i X=1 -- --config bumpy1m --steps 4
  run b1mt64k$i NH_TAIL=65536 -- --config bumpy1m --steps 4
done

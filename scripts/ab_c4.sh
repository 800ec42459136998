#!/usr/bin/env bash
# C4 chunking + tail A/B: A = optix-renderer_amd/lib, B = lib_alt; budget default vs one chunk per step
set -u
mkdir -p gpurun_out
run() {  # tag lib budget args...
  local tag=$1 lib=$2 bud=$3; shift 3
  if [ "$lib" = B ]; then export NH_LIB_PATH=$PWD/optix-renderer_amd/lib_alt/libnori_hip.so; else unset NH_LIB_PATH; fi
  if [ "$bud" != - ]; then export NH_WF_BUDGET_MB=$bud; else unset NH_WF_BUDGET_MB; fi
  timeout -k 10 300 python bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/ab_$tag.log; exit 99; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1])
print('$tag', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run c4A$i A - --config c4 --steps 8
  run c4B$i B - --config c4 --steps 8
  run c4A24g$i A 24576 --config c4 --steps 8
  run c4B24g$i B 24576 --config c4 --steps 8
done
run c2A A - --steps 16
run c2B B - --steps 16
run c2A24g A 24576 --steps 16

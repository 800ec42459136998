#!/usr/bin/env bash
# C4 knob sweep on the current library (env knobs: tail threshold, pools); C5 and C2 lines
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
for i in 1 2; do
  run c4def$i X=1 -- --config c4 --steps 8
  run c4t64k$i NH_TAIL=65536 -- --config c4 --steps 8
  run c4t1m$i NH_TAIL=1048576 -- --config c4 --steps 8
  run c4p3$i NH_POOLS=3 -- --config c4 --steps 8
done
run c5def X=1 -- --config c5 --steps 3 --warmup 1
run c5b8g NH_WF_BUDGET_MB=8192 -- --config c5 --steps 3 --warmup 1

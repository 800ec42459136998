#!/usr/bin/env bash
# path pools on the tail-bound C1 (1024^2 mirror + dielectric) and on C2 / C4
set -u
mkdir -p gpurun_out
run() {  # tag env... -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 "$@" > gpurun_out/sp_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/sp_$tag.log; exit 99; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/sp_$tag.log').read().strip().splitlines()[-1])
print('$tag', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run c1p2$i NH_POOLS=2 -- --config c1 --steps 8
  run c1p3$i NH_POOLS=3 -- --config c1 --steps 8
  run c1p4$i NH_POOLS=4 -- --config c1 --steps 8
done
run c2p2 NH_POOLS=2 -- --steps 16
run c2p3 NH_POOLS=3 -- --steps 16
run c4p3 NH_POOLS=3 -- --config c4 --steps 8
run c4p2 NH_POOLS=2 -- --config c4 --steps 8

#!/usr/bin/env bash
# A/B of the block-splat phase 2 (per-pixel vs column strips) on C2 / C4, same build, interleaved
set -u
mkdir -p gpurun_out
for i in 1 2; do
for cfg in c2 c4; do
  for v in "NH_SPLAT_STRIP=0" "NH_SPLAT_STRIP=1"; do
    env $v timeout -k 10 300 python bench.py --config $cfg --steps 8 --warmup 2 --no-cpu --no-denoise --traversal-1m-steps 0 > gpurun_out/ab_strip_${cfg}_${v}_$i.log 2>&1 || exit 99
    python3 -c "
import json
l=json.loads([x for x in open('gpurun_out/ab_strip_${cfg}_${v}_$i.log') if x.startswith('{')][0]); r=l['roofline']
print('$cfg $v $i', l['value'], l['ms_per_step'], 'splat/launch', r['splat_ms_per_launch'], 'dominant', r['avg_launch_ms'])"
  done
done
done

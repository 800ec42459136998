#!/usr/bin/env bash
# A/B of the splat + merge variants on C2 / C4 (same build): staged, fused 16x16 tiles, fused 32x32 tiles
set -u
mkdir -p gpurun_out
for cfg in c2 c4; do
  for v in "NH_SPLAT=staged" "NH_SPLAT_TILE=16" "NH_SPLAT_TILE=32"; do
    env $v timeout -k 10 300 python bench.py --config $cfg --steps 8 --warmup 2 --no-cpu --no-denoise --traversal-1m-steps 0 > gpurun_out/ab_splat_${cfg}_${v}.log 2>&1 || exit 99
    python3 -c "
import json
l=json.loads([x for x in open('gpurun_out/ab_splat_${cfg}_${v}.log') if x.startswith('{')][0]); r=l['roofline']
print('$cfg $v', l['value'], l['ms_per_step'], 'splat/launch', r['splat_ms_per_launch'], 'bounce', r['avg_launch_ms'])"
  done
done

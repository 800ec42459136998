#!/usr/bin/env bash
# A/B of the LDS copy of the top of the 4-wide tree (NH_TREE_TOP = nodes, 0 = off) on perf-1M and C3
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "trace or c3 or c5 or bumpy or wide" > gpurun_out/pytest_top.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_top.log
[ $rc -eq 0 ] || exit 99
for rep in 1 2; do
for v in 0 32 16; do
  NH_TREE_TOP=$v timeout -k 10 300 python bench.py --config bumpy1m --steps 4 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 > gpurun_out/ab_top_$v.log 2>&1 || exit 99
  python3 -c "
import json
l=json.loads([x for x in open('gpurun_out/ab_top_$v.log') if x.startswith('{')][0]); r=l['roofline']; e=r['stages']['extend']
print('bumpy1m top=$v', l['value'], 'extend', e['avg_launch_ms'], e['hbm_gbs'], round(e['hbm_gbs']/8000,4))"
done
done

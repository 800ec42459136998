#!/usr/bin/env bash
# Round 6: run-to-run spread of the C2 line on one box (final build), five back-to-back runs
set -u
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  log=gpurun_out/var_c2_$i.log
  timeout -k 10 300 python bench.py --config c2 --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 > $log 2>&1 || { echo "fail $i"; tail -5 $log; exit 99; }
  python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
print('c2 run $i', l['value'], l['ms_per_step'], 'dominant', r.get('avg_launch_ms'), 'splat', r.get('splat_ms_per_launch'))"
done

#!/usr/bin/env bash
# usage: scripts/sweep_env.sh VAR "v1 v2 ..." bench-args...   (one time-limited bench per value)
set -u
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
for v in $vals; do
  env "$var=$v" timeout -k 10 300 python bench.py "$@" > gpurun_out/sweep_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/sweep_$v.log; exit 99; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/sweep_$v.log').read().strip().splitlines()[-1])
r=d['roofline'] or {}
print('$var=$v', d['value'], d['ms_per_step'], json.dumps(r.get('stage_ms')), r.get('frac'))"
done

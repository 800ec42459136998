#!/usr/bin/env bash
# Interleaved A/B of one environment knob: scripts/ab_env.sh ROUNDS VAR "v1 v2 ..." bench-args...
set -u
n=$1; var=$2; vals=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python bench.py --no-cpu --no-calibrate "$@" > gpurun_out/abe_$v.$i.log 2>&1 || { echo "fail $v $i"; tail -3 gpurun_out/abe_$v.$i.log; exit 99; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/abe_$v.$i.log').read().strip().splitlines()[-1])
print('$var=$v', $i, d['value'], d['ms_per_step'])"
  done
done

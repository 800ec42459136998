#!/usr/bin/env bash
# Interleaved A/B of environment settings on one build: scripts/ab_env.sh ROUNDS "c2 c4" "NH_X=0 NH_X=1" [bench args]
# prints Msamples/s, ms/step, splat ms per launch, the dominant kernel's ms per launch and the serialized pass's
# tail stage (ms per launch, launches) per run
set -u
n=$1; cfgs=$2; vars=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for cfg in $cfgs; do
    for v in $vars; do
      log=gpurun_out/abe_${cfg}_${v}_$i.log
      env ${v//,/ } timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-denoise --traversal-1m-steps 0 "$@" > $log 2>&1 || { echo "fail $cfg $v"; tail -5 $log; exit 99; }
      python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
t=(r.get('stages') or {}).get('tail') or {}
print('$cfg $v $i', l['value'], l['ms_per_step'], 'splat/launch', r.get('splat_ms_per_launch'), 'dominant', r.get('avg_launch_ms'),
      'tail', t.get('avg_launch_ms'), t.get('launches'))"
    done
  done
done

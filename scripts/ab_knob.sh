#!/usr/bin/env bash
# Interleaved A/B of one environment knob over several bench configs (one bench process per cell).
# usage: scripts/ab_knob.sh KNOB "v1 v2 ..." "cfg:steps cfg:steps ..." [reps]
# prints one line per run: cfg knob=value Msamples/s
set -u
knob=$1; vals=$2; cfgs=$3; reps=${4:-1}
mkdir -p gpurun_out
for r in $(seq $reps); do
  for spec in $cfgs; do
    cfg=${spec%%:*}; steps=${spec#*:}
    for v in $vals; do
      log=gpurun_out/ab_${knob}_${v}_${cfg}_$r.log
      env $knob=$v timeout -k 10 240 python bench.py --config $cfg --steps $steps --no-cpu --traversal-1m-steps 0 --roofline-steps 0 > $log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$cfg $knob=$v rc=$rc"; tail -3 $log; exit 99; fi
      python3 -c "import json; l=json.loads(open('$log').readline()); print('$cfg', '$knob=$v', l['value'], l['ms_per_step'])"
    done
  done
done

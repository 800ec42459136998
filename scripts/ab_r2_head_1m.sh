#!/usr/bin/env bash
# Verdict r3 item 1: attribute the perf-1M traversal drop. Interleaved runs of round 2's bench + library
# (ab/r2: commit f8607b6, built in this container) and HEAD's on the bumpy-1M configuration, one box.
# usage: scripts/ab_r2_head_1m.sh ROUNDS [extra bench args]
set -u
n=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in r2 head; do
    b=ab/$v/bench.py
    timeout -k 10 300 python $b --config bumpy1m --steps 4 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 "$@" \
      > gpurun_out/ab1m_$v$i.log 2>&1 || { echo "fail $v$i"; tail -5 gpurun_out/ab1m_$v$i.log; exit 99; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ab1m_$v$i.log') if x.startswith('{')][0]); e=d['roofline']['stages']['extend']
print('$v$i', 'Msamples/s', d['value'], 'extend ms/launch', e['avg_launch_ms'], 'bytes/launch', e['global_bytes_per_launch'], 'frac', round(e['global_gbs']/8000, 4))"
  done
done

#!/usr/bin/env bash
# Verdict r3 item 1: attribute the perf-1M traversal drop and measure this round's traversal changes. Interleaved
# runs on the bumpy-1M configuration, one box: round 2's bench + library (ab/r2: commit f8607b6, built in this
# container), round 3's closing HEAD (ab/head), and the working tree (cur), optionally with env knobs (cur:K=V).
# usage: scripts/ab_r2_head_1m.sh ROUNDS "r2 head cur cur:NH_TRACE2=0" [extra bench args]
set -u
n=$1; variants=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in $variants; do
    name=${v%%:*}; knob=""; [ "$v" != "$name" ] && knob=${v#*:}
    b=bench.py; [ $name != cur ] && b=ab/$name/bench.py
    tag=$(echo "$v" | tr ':=,' '___')
    env $knob timeout -k 10 300 python $b --config bumpy1m --steps 4 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 \
      $( [ $name = cur ] && echo "--strong-spp 0 --no-extras" ) "$@" > gpurun_out/ab1m_$tag$i.log 2>&1 \
      || { echo "fail $v$i"; tail -5 gpurun_out/ab1m_$tag$i.log; exit 99; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ab1m_$tag$i.log') if x.startswith('{')][0]); st=d['roofline']['stages']
k='trace' if 'trace' in st else 'extend'; e=st[k]
sh=st.get('shadow', {})
tb = e['global_bytes_per_launch']*e['launches'] + sh.get('global_bytes_per_launch', 0)*sh.get('launches', 0)
tms = e['ms'] + sh.get('ms', 0)
print('$v$i', 'Msamples/s', d['value'], k, 'ms/launch', e['avg_launch_ms'], 'x', e['launches'], 'bytes/launch', e['global_bytes_per_launch'],
      'frac', round(e['global_gbs']/8000, 4), '| shadow ms', sh.get('ms'), 'frac', round(sh.get('global_gbs', 0)/8000, 4),
      '| both queries', round(tb/(tms*1e-3)/8e12, 4))"
  done
done

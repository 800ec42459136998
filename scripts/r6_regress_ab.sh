#!/usr/bin/env bash
# Round 6: C1 / C4 / megakernel against the round-5 closing build (wt/r5 = 3dc287c) and the normal-map commit (wt/nm =
# 02fc9e2), interleaved on one box; each build runs its own bench.py / binding / library from its worktree.
set -u
mkdir -p gpurun_out
root=$PWD
for i in 1 2; do
  for cfg in c1 c4; do
    for b in r5 nm cur; do
      d=$root/wt/$b; [ $b = cur ] && d=$root
      log=$root/gpurun_out/rg_${cfg}_${b}_$i.log
      (cd $d && timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 > $log 2>&1) || { echo "fail $cfg $b"; tail -5 $log; exit 99; }
      python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
t=(r.get('stages') or {}).get('tail') or {}
print('$cfg $b $i', l['value'], l['ms_per_step'], 'splat', r.get('splat_ms_per_launch'), 'dominant', r.get('avg_launch_ms'), 'tail', t.get('avg_launch_ms'))"
    done
  done
done
for b in r5 cur; do
  d=$root/wt/$b; [ $b = cur ] && d=$root
  log=$root/gpurun_out/rg_mk_${b}.log
  (cd $d && timeout -k 10 300 python bench.py --config c2 --mode megakernel --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 > $log 2>&1) || { echo "fail mk $b"; tail -5 $log; exit 99; }
  python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0])
print('megakernel $b', l['value'], l['ms_per_step'])"
done

#!/usr/bin/env bash
# Round 6, verdict r5 item 4: the pair splat (NH_SPLAT_PAIR) against the one-launch staged splat + merge.
# Interleaved C2 / C4 runs on one box, then one kernel-trace pass per mode (C2, one pool) for per-kernel durations.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in c2 c4; do
    for v in "lib NH_SPLAT_PAIR=0" "lib NH_SPLAT_PAIR=1" "lib_late NH_SPLAT_PAIR=1"; do
      set -- $v
      if [ $1 = lib ]; then unset NH_LIB_PATH; else export NH_LIB_PATH=$PWD/optix-renderer_amd/$1/libnori_hip.so; fi
      log=gpurun_out/pab_${cfg}_$1_$2_$i.log
      env $2 timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-denoise --traversal-1m-steps 0 > $log 2>&1 || { echo "fail $cfg $v"; tail -5 $log; exit 99; }
      python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
print('$cfg $1 $2 $i', l['value'], l['ms_per_step'], 'splat/launch', r.get('splat_ms_per_launch'), 'dominant', r.get('avg_launch_ms'))"
    done
  done
done
unset NH_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 0 1; do
  env NH_SPLAT_PAIR=$p timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_trace$p -o run -- python3 bench.py --config c2 --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --roofline-steps 0 --pools 1 --steps 4 --warmup 1 --strong-spp 0 --no-extras > gpurun_out/pab_trace$p.log 2>&1 || { echo "trace $p failed"; exit 99; }
  python3 - <<PY
import csv,glob
f=glob.glob('gpurun_out/pab_trace$p/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('splat','merge')): print('$p', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
done

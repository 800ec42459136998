#!/usr/bin/env bash
# Round 6 (second call): the NMAP = false full bodies and the path_mis-only megakernel against the round-5 build
# (wt/r5), after the GPU suite on the new build
set -u
mkdir -p gpurun_out
root=$PWD
scripts/gpu_step.sh 600 gpurun_out/pytest_nmap.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_nmap.log && ! grep -q " failed" gpurun_out/pytest_nmap.log || { tail -30 gpurun_out/pytest_nmap.log; exit 98; }
grep -E "passed|failed" gpurun_out/pytest_nmap.log | tail -1
run() {  # tag dir args...
  local tag=$1 d=$2; shift 2
  local log=$root/gpurun_out/nm2_$tag.log
  (cd $d && timeout -k 10 300 python bench.py --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 "$@" > $log 2>&1) || { echo "fail $tag"; tail -5 $log; exit 99; }
  python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
print('$tag', l['value'], l['ms_per_step'], 'dominant', r.get('avg_launch_ms'))"
}
for i in 1 2; do
  for cfg in c1 c4 c2; do
    run ${cfg}_r5_$i $root/wt/r5 --config $cfg || exit 99
    run ${cfg}_cur_$i $root --config $cfg || exit 99
  done
  run mk_r5_$i $root/wt/r5 --config c2 --mode megakernel || exit 99
  run mk_cur_$i $root --config c2 --mode megakernel || exit 99
done

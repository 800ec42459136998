#!/usr/bin/env bash
# Round 6: is the C1 / C4 / megakernel regression since round 5 the normal-map code in hit_info? lib (current) vs
# lib_nonmap (-DNH_AB_NO_NMAP: the normal-map branch compiled out; attribution only) vs the round-5 build (wt/r5)
set -u
mkdir -p gpurun_out
root=$PWD
run() {  # tag dir libpath args...
  local tag=$1 d=$2 lp=$3; shift 3
  local log=$root/gpurun_out/nm_$tag.log
  if [ -n "$lp" ]; then export NH_LIB_PATH=$lp; else unset NH_LIB_PATH; fi
  (cd $d && timeout -k 10 300 python bench.py --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 "$@" > $log 2>&1) || { echo "fail $tag"; tail -5 $log; exit 99; }
  python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0]); r=l['roofline'] or {}
print('$tag', l['value'], l['ms_per_step'], 'dominant', r.get('avg_launch_ms'))"
}
for i in 1 2; do
  for cfg in c1 c4; do
    run ${cfg}_r5_$i $root/wt/r5 "" --config $cfg || exit 99
    run ${cfg}_cur_$i $root "" --config $cfg || exit 99
    run ${cfg}_nonmap_$i $root $root/optix-renderer_amd/lib_nonmap/libnori_hip.so --config $cfg || exit 99
  done
  run mk_r5_$i $root/wt/r5 "" --config c2 --mode megakernel || exit 99
  run mk_cur_$i $root "" --config c2 --mode megakernel || exit 99
  run mk_nonmap_$i $root $root/optix-renderer_amd/lib_nonmap/libnori_hip.so --config c2 --mode megakernel || exit 99
done

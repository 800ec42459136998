#!/usr/bin/env bash
# Round 6: the path_mis-only megakernel (496 B scratch at 4 waves/SIMD) at NH_PATH_WAVES=2 vs the default 4, C2
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for w in 4 2; do
    log=gpurun_out/mkw_${w}_$i.log
    NH_PATH_WAVES=$w timeout -k 10 300 python bench.py --config c2 --mode megakernel --no-cpu --no-denoise --traversal-1m-steps 0 --no-extras --strong-spp 0 > $log 2>&1 || { echo "fail $w"; tail -5 $log; exit 99; }
    python3 -c "
import json
l=json.loads([x for x in open('$log') if x.startswith('{')][0])
print('NH_PATH_WAVES=$w $i', l['value'], l['ms_per_step'])"
  done
done

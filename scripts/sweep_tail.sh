#!/usr/bin/env bash
set -u
mkdir -p gpurun_out
for t in 1048576 262144 131072 65536; do
  NH_TAIL=$t timeout -k 10 300 python bench.py --config c4 --no-cpu --no-calibrate --steps 2 > gpurun_out/tail_$t.log 2>&1 || { echo fail; exit 99; }
  python3 -c "
import json
l=json.loads(open('gpurun_out/tail_$t.log').read().strip().splitlines()[-1]); print($t, l['value'], l['ms_per_step'])"
done

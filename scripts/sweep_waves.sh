#!/usr/bin/env bash
# occupancy sweep of the path megakernel on the C2 bench workload
for w in 1 2 3 4; do
  NH_PATH_WAVES=$w timeout -k 10 120 python bench.py --no-cpu --steps 8 --warmup 1 > gpurun_out/sweep_w$w.json 2>&1 || exit 99
  python -c "import json;d=json.load(open('gpurun_out/sweep_w$w.json'));print('waves=$w', d['value'], 'Msamples/s', d['roofline']['avg_launch_ms'], 'ms/launch', 'splat', d['roofline']['splat_ms_per_launch'])"
done

#!/usr/bin/env bash
# kernel-trace timeline of a short C1 / C4 bench (for the tail overlap analysis) + the default bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in c1 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$cfg -o run -- python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-denoise --no-calibrate --traversal-1m-steps 0 --roofline-steps 0 > gpurun_out/trace_$cfg.log 2>&1 || exit 99
done
timeout -k 10 400 python bench.py > gpurun_out/bench_r3c.log 2>&1 || exit 99
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 > gpurun_out/bench_r3c_c5.log 2>&1 || exit 99
echo done

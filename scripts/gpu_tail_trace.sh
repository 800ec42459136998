#!/usr/bin/env bash
# kernel timelines of C1 with in-place and with asynchronous tails
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1; do
  NH_TAIL_ASYNC=$a timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trt_$a -o run -- python3 bench.py --config c1 --no-cpu --no-denoise --traversal-1m-steps 0 --steps 8 --warmup 2 --roofline-steps 0 > gpurun_out/trt_$a.log 2>&1 || exit 99
  head -c 300 gpurun_out/trt_$a.log; echo
done

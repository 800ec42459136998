#!/usr/bin/env bash
# Kernel trace of the timed bench steps (no calibration / roofline passes) and the GPU-busy timeline summary.
# usage: scripts/trace_timeline.sh TAG bench-args...  -> gpurun_out/tl_TAG/{timeline.txt, run_kernel_stats.csv}
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/tl_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --no-cpu \
  --no-calibrate --roofline-steps 0 --strong-spp 0 --no-extras --no-denoise --traversal-1m-steps 0 "$@" > $out/bench.log 2>&1 \
  || { echo "trace failed"; tail -5 $out/bench.log; exit 99; }
f=$(find $out -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" 0.2 > $out/timeline.txt
head -3 $out/timeline.txt
grep "^{" $out/bench.log | cut -c1-200

#!/usr/bin/env bash
# kernel-trace (rocpd db) of one bench configuration: scripts/prof_trace.sh TAG bench-args...
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$tag
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu --no-calibrate "$@" > gpurun_out/prof_$tag/bench.log 2>&1 || { tail -5 gpurun_out/prof_$tag/bench.log; exit 99; }
grep "^{" gpurun_out/prof_$tag/bench.log | cut -c1-300

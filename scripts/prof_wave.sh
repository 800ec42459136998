#!/usr/bin/env bash
# kernel-trace profile of the wavefront pipeline on c2 (2 steps)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_wave
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wave -o wave -- python3 bench.py --mode wavefront --steps 2 --warmup 0 --no-cpu --no-calibrate > gpurun_out/prof_wave/bench.log 2>&1 || exit 99
find gpurun_out/prof_wave -name "*.csv" | head

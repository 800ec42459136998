#!/usr/bin/env bash
# Round evidence for the default config: smoke + GPU suite + bench + kernel trace + PMC, then the
# PMC traffic of the bumpy-1M traversal kernel.
set -u
tag=$1
scripts/gpu_full.sh $tag || exit 99
scripts/pmc.sh ${tag}_bumpy --config bumpy1m > /dev/null || exit 99
scripts/gpu_step.sh 300 gpurun_out/bench_${tag}_bumpy.log python bench.py --config bumpy1m --no-cpu --steps 4 || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_${tag}_bumpy -o run -- python3 bench.py --no-cpu --config bumpy1m --steps 4 > gpurun_out/trace_${tag}_bumpy.log 2>&1 || exit 99
tail -1 gpurun_out/bench_${tag}_bumpy.log

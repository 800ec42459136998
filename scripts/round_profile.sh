#!/usr/bin/env bash
# GPU parity tests, the default bench line, its rocprofv3 kernel-trace summary and the PMC passes.
# usage: scripts/round_profile.sh TAG [extra bench args...]
set -u
tag=$1; shift
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 99
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 98; }
scripts/gpu_step.sh 400 gpurun_out/bench_$tag.log python bench.py "$@" || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu "$@" > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
scripts/pmc.sh $tag "$@" > /dev/null || exit 99
tail -1 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/bench_$tag.log
grep -h "wf_\|nh_" gpurun_out/trace_$tag/*kernel_stats.csv | cut -c1-200

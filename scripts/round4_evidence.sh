#!/usr/bin/env bash
# Round-4 evidence, part 1: smoke, GPU suite, default bench line. usage: scripts/round4_evidence.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -30 gpurun_out/pytest_$tag.log; exit 98; }
scripts/gpu_step.sh 500 gpurun_out/bench_$tag.log python bench.py || exit 99
tail -1 gpurun_out/pytest_$tag.log
cat gpurun_out/smoke_$tag.log

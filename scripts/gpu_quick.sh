#!/usr/bin/env bash
# Smoke + GPU suite + default bench line: scripts/gpu_quick.sh TAG [pytest -k expression]
set -u
tag=$1; k=${2:-}
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
if [ -n "$k" ]; then
  scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -k "$k" || exit 99
else
  scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
fi
tail -3 gpurun_out/pytest_$tag.log
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { grep -E "FAIL|Error" gpurun_out/pytest_$tag.log | head -20; exit 98; }
scripts/gpu_step.sh 400 gpurun_out/bench_$tag.log python bench.py || exit 99
grep "^{" gpurun_out/bench_$tag.log | cut -c1-400
cat gpurun_out/smoke_$tag.log

#!/usr/bin/env bash
# Round-3 evidence: smoke, GPU suite, default bench line, rocprofv3 kernel trace + stats of the same command,
# C1 / C3 / C4 / C5 bench lines. usage: scripts/round3_evidence.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/gpu_step.sh 500 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -30 gpurun_out/pytest_$tag.log; exit 98; }
scripts/gpu_step.sh 400 gpurun_out/bench_$tag.log python bench.py || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
for cfg in c1 c4 c3 c5; do
  steps=8; [ $cfg = c5 ] && steps=3; [ $cfg = c3 ] && steps=2
  scripts/gpu_step.sh 300 gpurun_out/bench_${tag}_$cfg.log python bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 || exit 99
done
tail -1 gpurun_out/pytest_$tag.log
cat gpurun_out/smoke_$tag.log

#!/usr/bin/env bash
# Round-4 evidence, part 2: rocprofv3 kernel trace + stats of the default bench command, C1 / C4 / C3 / C5 lines.
# usage: scripts/round4_evidence2.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
for cfg in c1 c4 c3 c5; do
  steps=8; [ $cfg = c5 ] && steps=3; [ $cfg = c3 ] && steps=2
  scripts/gpu_step.sh 300 gpurun_out/bench_${tag}_$cfg.log python bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 --strong-spp 0 --no-extras || exit 99
done
grep -h '^{' gpurun_out/bench_${tag}_*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['config'], json.loads(l)['value']) for l in sys.stdin]"

#!/usr/bin/env bash
# Second half of scripts/evidence.sh: bench lines of every configuration and the kernel trace + stats of the default
# bench command (run after evidence_a.sh and after profiles/pmc_traffic.json holds its records).
# usage: scripts/evidence_b.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
scripts/gpu_step.sh 500 gpurun_out/bench_$tag.log python bench.py || exit 99
for cfg in c1 c3 c4 c5 bumpy1m; do
  scripts/gpu_step.sh 400 gpurun_out/bench_${tag}_$cfg.log python bench.py --config $cfg --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 || exit 99
done
grep -h "^{" gpurun_out/bench_$tag.log gpurun_out/bench_${tag}_*.log > gpurun_out/bench_lines_$tag.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
python3 -c "
import json
for l in open('gpurun_out/bench_lines_$tag.jsonl'):
    d = json.loads(l); r = d.get('roofline') or {}
    print(d['config'].get('config'), d['value'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'limiter', bool(r.get('limiter')))"

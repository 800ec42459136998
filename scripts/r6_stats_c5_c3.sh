#!/usr/bin/env bash
# Round 6: kernel trace + stats of the C5 and C3 bench commands on the final build
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c5 c3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_f_$cfg -o run -- python3 bench.py --config $cfg --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 > gpurun_out/trace_f_$cfg.log 2>&1 || { echo "trace $cfg failed"; tail -5 gpurun_out/trace_f_$cfg.log; exit 99; }
  grep -h '^{' gpurun_out/trace_f_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'])"
done

#!/usr/bin/env bash
# Round 6, verdict r5 item 4 (second call): splat parity, the pair splat's kernel trace and PMC bytes (C2, one pool),
# and NH_SPLAT_PAIR=0 / 1 on C1 / C3 / C5
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "fused_splat" > gpurun_out/pab2_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/pab2_tests.log; exit 99; }
tail -1 gpurun_out/pab2_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab2_trace1 -o run -- python3 bench.py --config c2 --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --roofline-steps 0 --pools 1 --steps 4 --warmup 1 --strong-spp 0 --no-extras > gpurun_out/pab2_trace1.log 2>&1 || { echo "trace failed"; exit 99; }
python3 - <<PY
import csv,glob
f=glob.glob('gpurun_out/pab2_trace1/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('splat','merge')): print('trace', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
bash scripts/pmc_splat.sh pair1 NH_SPLAT_PAIR=1 || exit 99
bash scripts/pmc_splat.sh pair0 NH_SPLAT_PAIR=0 || exit 99
bash scripts/ab_env.sh 1 "c1 c3 c5" "NH_SPLAT_PAIR=0 NH_SPLAT_PAIR=1"

#!/usr/bin/env bash
# direct interior pixels in the tab splat: parity, A/B, kernel times
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_splat or parity_cbox or pipelined or deterministic" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_direct.log 2>&1 || { tail -30 gpurun_out/t_direct.log; exit 99; }
tail -1 gpurun_out/t_direct.log
scripts/ab_env.sh 2 "c2 c4" "NH_SPLAT_DIRECT=0 NH_SPLAT_DIRECT=1" --steps 8 --warmup 2 || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1; do
  NH_SPLAT_DIRECT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trd$v -o run -- python3 bench.py --config c2 --pools 1 --no-cpu --no-denoise --traversal-1m-steps 0 --steps 3 --warmup 1 > gpurun_out/trd$v.log 2>&1 || exit 99
  echo "== NH_SPLAT_DIRECT=$v"; grep -h "splat\|merge" gpurun_out/trd$v/run_kernel_stats.csv | cut -d, -f1-4,6,7
done

#!/usr/bin/env bash
# tab splat: rounds per workgroup (NH_SPLAT_ROUNDS 1/2/4/8), parity + kernel times on C2 (one pool)
set -u
mkdir -p gpurun_out
for r in 1 2 8; do
  NH_SPLAT_ROUNDS=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_splat or deterministic" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_rounds$r.log 2>&1 || { tail -30 gpurun_out/t_rounds$r.log; exit 99; }
  tail -1 gpurun_out/t_rounds$r.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 4 8; do
  NH_SPLAT_ROUNDS=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trr$r -o run -- python3 bench.py --config c2 --pools 1 --no-cpu --no-denoise --traversal-1m-steps 0 --steps 3 --warmup 1 > gpurun_out/trr$r.log 2>&1 || exit 99
  echo "== NH_SPLAT_ROUNDS=$r"; grep -h "splat\|merge" gpurun_out/trr$r/run_kernel_stats.csv | cut -d, -f1-4,6,7
done
cd "$GRAFT_REPO_ROOT"
scripts/ab_env.sh 1 "c2 c4" "NH_SPLAT_ROUNDS=4 NH_SPLAT_ROUNDS=2 NH_SPLAT_ROUNDS=1" --steps 8 --warmup 2 || exit 99

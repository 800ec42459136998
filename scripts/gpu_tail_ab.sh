#!/usr/bin/env bash
# async tails A/B on the specular configs (+ parity tests of the touched paths), splat/merge kernel times
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_splat or async_tails or variants or pipelined or parity_cbox" -x -q --timeout 250 --timeout-method thread > gpurun_out/t_tail.log 2>&1 || { tail -30 gpurun_out/t_tail.log; exit 99; }
tail -1 gpurun_out/t_tail.log
scripts/ab_env.sh 1 "c1 c4 c2" "NH_TAIL_ASYNC=0 NH_TAIL_ASYNC=1 NH_TAIL_ASYNC=1,NH_WF_BUDGET_MB=8192" --steps 8 --warmup 2 || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trm -o run -- python3 bench.py --config c2 --pools 1 --no-cpu --no-denoise --traversal-1m-steps 0 --steps 3 --warmup 1 > gpurun_out/trm.log 2>&1 || exit 99
grep -h "splat\|merge" gpurun_out/trm/run_kernel_stats.csv | cut -d, -f1-4,6,7

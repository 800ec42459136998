set -u
mkdir -p gpurun_out
bash scripts/ab_env.sh 2 "c2" "NH_TAIL_RR_WAVES=4 NH_TAIL_RR_WAVES=1 NH_TAIL=32768 NH_TAIL=131072" --strong-spp 0 --no-extras || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_r5c2 -o run -- python3 bench.py --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 > gpurun_out/trace_r5c2.log 2>&1 || { tail -5 gpurun_out/trace_r5c2.log; exit 99; }
head -12 gpurun_out/trace_r5c2/run_kernel_stats.csv | cut -c1-200

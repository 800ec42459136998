# round 4: rocprofv3 kernel trace + stats of the C1 and C4 bench commands (tail kernels beside the pools' bounces)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c1 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_r4_$cfg -o run -- python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 --strong-spp 0 --no-extras > gpurun_out/trace_r4_$cfg.log 2>&1 || { echo "trace $cfg failed"; tail -5 gpurun_out/trace_r4_$cfg.log; exit 99; }
done
echo traces done

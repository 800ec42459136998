#!/usr/bin/env bash
# kernel durations of the splat variants, one pool (kernels alone on the GPU)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "NH_SPLAT_DEBUG=0" "NH_SPLAT_DEBUG=15" "NH_SPLAT_DEBUG=3" "NH_SPLAT_FUSED=0"; do
  export $v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trs_$v -o run -- python3 bench.py --config c2 --pools 1 --no-cpu --no-denoise --traversal-1m-steps 0 --steps 3 --warmup 1 > gpurun_out/trs_$v.log 2>&1 || exit 99
  unset ${v%%=*}
  echo "== $v"; grep -h "splat\|merge" gpurun_out/trs_$v/run_kernel_stats.csv | cut -d, -f1-4,6,7
done

#!/usr/bin/env bash
# Host-trap PC sampling of one kernel in one bench configuration (rocprofv3 beta): which instructions the waves
# sit on. usage: scripts/pc_sample.sh TAG KERNEL_REGEX bench-args...  -> gpurun_out/pcs_TAG/
set -u
tag=$1; kre=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pcs_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 --kernel-include-regex "$kre" --output-format csv -d $out -o run -- \
  python3 bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --strong-spp 0 --no-extras "$@" \
  > $out/bench.log 2>&1
rc=$?
echo "pc sampling rc=$rc"
find $out -name "*.csv" | head
exit $rc

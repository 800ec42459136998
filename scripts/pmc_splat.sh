#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for the C2 splat + merge, one pool.
# usage: scripts/pmc_splat.sh TAG [ENV=VAL ...]  -> gpurun_out/pmcs_TAG/summary.txt
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmcs_$tag
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  env "$@" timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --config c2 --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --roofline-steps 0 --pools 1 --steps 2 --warmup 0 --strong-spp 0 --no-extras > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 99; }
done
python3 scripts/pmc_summary.py $out | grep -E "splat|merge" > $out/summary.txt; cat $out/summary.txt

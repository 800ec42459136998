#!/usr/bin/env bash
# instruction-fetch PMC of one bench configuration (one counter group per rocprofv3 run, kernel-trace only)
# usage: scripts/pmc_icache.sh TAG bench-args...  -> gpurun_out/pmci_TAG/p<i>/...counter_collection.csv
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmci_$tag
mkdir -p $out
i=0
for grp in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --roofline-steps 0 --pools 1 --steps 2 --warmup 0 --strong-spp 0 --no-extras "$@" > $out/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $out/p$i.log; exit 99; }
done
python3 scripts/pmc_summary.py $out | grep -E "bounce_rr|tail_rr|splat" > $out/summary.txt; cat $out/summary.txt

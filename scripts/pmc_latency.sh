#!/usr/bin/env bash
# Where a kernel's waves wait: instruction mix by memory type and the in-flight levels (Little's law: average
# latency = level / instructions) in separate rocprofv3 --pmc passes, kernel-trace only.
# usage: scripts/pmc_latency.sh TAG bench-args...  -> gpurun_out/pmcl_TAG/summary.txt
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmcl_$tag
mkdir -p $out
i=0
for grp in "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_INST_LEVEL_VMEM" "SQ_INST_LEVEL_LDS" "SQ_INST_LEVEL_SMEM" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu --no-calibrate \
    --traversal-1m-steps 0 --roofline-steps 0 --strong-spp 0 --no-extras --no-denoise --steps 2 --warmup 0 "$@" > $out/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) failed rc=$rc"; tail -3 $out/p$i.log
    # a killed / crashed pass ends the session; a counter the tool rejects does not
    if [ $rc -ge 124 ]; then exit 99; fi
  fi
done
python3 scripts/pmc_summary.py $out > $out/summary.txt; grep -E "bounce_rr|splat_tab" $out/summary.txt

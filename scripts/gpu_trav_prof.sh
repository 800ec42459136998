#!/usr/bin/env bash
# Traversal profile of one config: counter list, kernel trace (VGPRs, durations), SQ/LDS PMC passes.
set -u
cfg=${1:-bumpy1m}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
out=gpurun_out/tprof_$cfg
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --config $cfg --steps 2 --warmup 1 > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 99; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu --no-calibrate --config $cfg --steps 1 --warmup 0 --pools 1 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
done
python3 scripts/pmc_summary.py $out > $out/summary.txt; grep -h "wf_trace_pt\|wf_shade" $out/summary.txt | cut -c1-160

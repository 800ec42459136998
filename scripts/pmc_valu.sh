#!/usr/bin/env bash
# PMC passes for the issue / divergence diagnosis of one bench configuration (one counter group per
# rocprofv3 run, kernel-trace only; no pass exceeds the gfx950 per-block slots: SQ 8, TCC 4, GRBM 2).
# usage: scripts/pmc_valu.sh TAG bench-args...   -> gpurun_out/pmcv_TAG/p<i>/...counter_collection.csv
# PMC_PASSES="1 4 5 6 7" limits the run to those passes (default: all eight; 8 = LDS conflicts / waits)
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmcv_$tag
mkdir -p $out
i=0
for grp in "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
           "VALUBusy VALUUtilization" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAVE_CYCLES"; do
  i=$((i+1))
  case " ${PMC_PASSES:-1 2 3 4 5 6 7 8} " in *" $i "*) ;; *) continue ;; esac
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu --no-calibrate --no-denoise --traversal-1m-steps 0 --roofline-steps 0 --pools 1 "$@" > $out/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $out/p$i.log; exit 99; }
done
python3 scripts/pmc_summary.py $out > $out/summary.txt && echo "pmc $tag done"

#!/usr/bin/env bash
# VALU issue ceiling: tools/bin/valu_issue's sweep (fp32 FMA, packed FMA, fp64 FMA, sqrt, int mix at
# 1/2/4/8 waves per SIMD) timed with HIP events, then one rocprofv3 PMC pass for the counter view.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/valu_issue
mkdir -p $out
timeout -k 10 120 tools/bin/valu_issue > $out/events.jsonl 2>&1 || { echo "valu_issue failed"; cat $out/events.jsonl; exit 99; }
cat $out/events.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $out/pmc -o run -- tools/bin/valu_issue > $out/pmc.log 2>&1 || { echo "pmc pass failed"; tail -5 $out/pmc.log; exit 99; }
python3 scripts/valu_issue_summary.py $out > $out/summary.txt && cat $out/summary.txt

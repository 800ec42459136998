#!/usr/bin/env bash
# Round evidence: smoke, GPU suite, default bench line, rocprofv3 kernel trace of the same command,
# PMC passes (HBM bytes, VALU / wait counters, L2) for C2 and perf-1M, and the traffic summary.
# usage: scripts/round_evidence.sh TAG
set -u
tag=$1
mkdir -p gpurun_out
S="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
scripts/gpu_step.sh 150 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/gpu_step.sh 500 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread || exit 99
grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { tail -30 gpurun_out/pytest_$tag.log; exit 98; }
scripts/gpu_step.sh 400 gpurun_out/bench_$tag.log python bench.py || exit 99
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --no-cpu > gpurun_out/trace_$tag.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace_$tag.log; exit 99; }
scripts/pmc_groups.sh ${tag}_c2 "FETCH_SIZE" "WRITE_SIZE" "$S" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" -- --config c2 > /dev/null || exit 99
scripts/pmc_groups.sh ${tag}_bumpy "FETCH_SIZE" "WRITE_SIZE" "$S" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" -- --config bumpy1m > /dev/null || exit 99
tail -1 gpurun_out/pytest_$tag.log
cat gpurun_out/smoke_$tag.log

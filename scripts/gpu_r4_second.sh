# round 4, second GPU session: the full GPU suite, then A/B of this round's kernel changes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4b.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -5 gpurun_out/pytest_gpu_r4b.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4b.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c1 2 "head cur cur:NH_TAIL_RR_WAVES=1" > gpurun_out/ab_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab_c1.txt
bash scripts/ab_variants.sh c4 1 "head cur cur:NH_TAIL_RR_WAVES=1" > gpurun_out/ab_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab_c4.txt
bash scripts/ab_variants.sh c2 2 "head cur" > gpurun_out/ab_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab_c2.txt
bash scripts/ab_variants.sh bumpy1m 2 "r2 head cur cur:NH_TRACE2=0" > gpurun_out/ab_1m.txt 2>&1; echo "ab 1m rc=$?"; cat gpurun_out/ab_1m.txt

# round 4, third GPU session: GPU suite, then the tail / bounce A/B (cooperative finish, register budget, uv skip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4c.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4c.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4c.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c1 2 "head cur cur:NH_TAIL_COOP=1 cur:NH_TAIL_RR_WAVES=1 cur:NH_TAIL_RR_WAVES=1,NH_TAIL_COOP=1" > gpurun_out/ab3_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab3_c1.txt
bash scripts/ab_variants.sh c4 1 "head cur cur:NH_TAIL_COOP=1 cur:NH_TAIL_RR_WAVES=1" > gpurun_out/ab3_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab3_c4.txt
bash scripts/ab_variants.sh c2 2 "head cur" > gpurun_out/ab3_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab3_c2.txt
bash scripts/ab_variants.sh bumpy1m 1 "cur cur:NH_TREE_TOP=0" > gpurun_out/ab3_1m.txt 2>&1; echo "ab 1m rc=$?"; cat gpurun_out/ab3_1m.txt

# round 4, fourth GPU session: GPU suite, tail / bounce A/B with 8 hardware queues, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4d.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4d.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4d.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c1 2 "head cur cur:NH_TAIL_RR_WAVES=1" > gpurun_out/ab4_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab4_c1.txt
bash scripts/ab_variants.sh c4 2 "head cur cur:NH_TAIL_RR_WAVES=1" > gpurun_out/ab4_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab4_c4.txt
bash scripts/ab_variants.sh c2 2 "head cur" > gpurun_out/ab4_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab4_c2.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r4d.jsonl 2> gpurun_out/bench_default_r4d.err; echo "bench rc=$?"; tail -c 3000 gpurun_out/bench_default_r4d.jsonl

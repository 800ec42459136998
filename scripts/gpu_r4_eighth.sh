# round 4, eighth GPU session: RGB-only sample records (the splat recomputes the jitter), core + band staging layout,
# lead splat workgroup: full GPU suite, C2 A/B against round 3's HEAD, splat PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4h.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4h.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_r4h.log | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 2 "head cur cur:NH_SPLAT_ROUNDS=8 cur:NH_SPLAT_LEAD=0" > gpurun_out/ab8_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab8_c2.txt
bash scripts/pmc_splat.sh r4j4 && bash scripts/pmc_splat.sh r4j8 NH_SPLAT_ROUNDS=8

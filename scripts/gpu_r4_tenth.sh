# round 4, tenth GPU session: jitter recomputed vs stored (NH_SPLAT_JITTER=stored), pair planes in the tab splat:
# splat parity, C2 A/B against round 3's HEAD, splat PMC of both jitter modes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or wavefront_matches" > gpurun_out/pytest_gpu_r4j.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4j.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_r4j.log | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 3 "head cur cur:NH_SPLAT_JITTER=stored" > gpurun_out/ab10_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab10_c2.txt
bash scripts/pmc_splat.sh r4p8 && bash scripts/pmc_splat.sh r4p8s NH_SPLAT_JITTER=stored

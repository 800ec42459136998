# round 4, seventh GPU session: splat parity (lead workgroup direct, aligned staging rows), C2 A/B, splat PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or isolated or wavefront_matches or variants" > gpurun_out/pytest_gpu_r4g.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4g.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_r4g.log | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 2 "head cur cur:NH_SPLAT_ROUNDS=8 cur:NH_SPLAT_LEAD=0" > gpurun_out/ab7_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab7_c2.txt
bash scripts/pmc_splat.sh r4lead4 && bash scripts/pmc_splat.sh r4lead8 NH_SPLAT_ROUNDS=8 && bash scripts/pmc_splat.sh r4nolead NH_SPLAT_LEAD=0

# round 4, ninth GPU session: jitter formed with the record prefetch, 8 rounds per splat workgroup (lead = half the
# rounds): splat / wavefront parity, C2 A/B against round 3's HEAD, splat PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or isolated or wavefront_matches or variants" > gpurun_out/pytest_gpu_r4i.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4i.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_r4i.log | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 3 "head cur cur:NH_SPLAT_LEAD=0" > gpurun_out/ab9_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab9_c2.txt
bash scripts/pmc_splat.sh r4k8

# round 4, sixth GPU session: isolated-sphere closest hits (parity first), then C1 / C4 / C2 A/B against round 3's HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4f.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4f.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_r4f.log | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c1 2 "head cur cur:NH_ISO_SPHERE=0" > gpurun_out/ab6_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab6_c1.txt
bash scripts/ab_variants.sh c4 2 "head cur cur:NH_ISO_SPHERE=0" > gpurun_out/ab6_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab6_c4.txt
bash scripts/ab_variants.sh c2 2 "head cur" > gpurun_out/ab6_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab6_c2.txt

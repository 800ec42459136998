# round 4, fifth GPU session: parity (NEE-first shade body, tail register default, cooperative-phase clocks),
# C2 / C1 A/B against round 3's HEAD with the cooperative bounces' latency in the tail profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_textures.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4e.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -3 gpurun_out/pytest_gpu_r4e.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4e.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 3 "head cur" > gpurun_out/ab5_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab5_c2.txt
bash scripts/ab_variants.sh c1 2 "head cur" > gpurun_out/ab5_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab5_c1.txt

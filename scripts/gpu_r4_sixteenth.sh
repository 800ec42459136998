# round 4, sixteenth GPU session: lean wf_bounce_rr (no light-sample skip, isolated-sphere test or texture lookup) for scenes
# with no mirror / dielectric BSDF (template SKIP): parity, C2 and C1 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_textures.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4l.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -2 gpurun_out/pytest_gpu_r4l.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4l.log | head -5
[ $rc -ne 0 ] && exit $rc
L=NH_LIB_PATH=optix-renderer_amd
bash scripts/ab_variants.sh c2 3 "head cur cur:$L/vC/libnori_hip.so" > gpurun_out/ab16_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab16_c2.txt
bash scripts/ab_variants.sh c1 2 "head cur" > gpurun_out/ab16_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab16_c1.txt

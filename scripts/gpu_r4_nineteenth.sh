# round 4, nineteenth GPU session: persistent splat grid (NH_SPLAT_WGS: the splat holds fewer CUs' LDS while the other
# pool's bounce kernels run): splat parity, C2 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "splat" > gpurun_out/pytest_gpu_r4o.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -2 gpurun_out/pytest_gpu_r4o.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4o.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 3 "cur cur:NH_SPLAT_WGS=128 cur:NH_SPLAT_WGS=256 cur:NH_SPLAT_WGS=512" > gpurun_out/ab19_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab19_c2.txt

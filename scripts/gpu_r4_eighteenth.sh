# round 4, eighteenth GPU session: the jitter mode as a template parameter of the tab splat: splat and
# wavefront parity, C2 A/B against round 3's HEAD and the stored jitter
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or wavefront_matches or variants" > gpurun_out/pytest_gpu_r4n.log 2>&1; rc=$?; echo "gpu parity rc=$rc"; tail -2 gpurun_out/pytest_gpu_r4n.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r4n.log | head -5
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_variants.sh c2 3 "head cur cur:NH_SPLAT_JITTER=stored" > gpurun_out/ab18_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab18_c2.txt
bash scripts/pmc_splat.sh r4tmpl

#!/usr/bin/env bash
# Round 6: wf_shade<.., NMAP = false> (deep BVHs, scenes without normal maps) vs the build before it (lib_prev);
# deep-BVH GPU tests first
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 400 gpurun_out/pytest_shade_nmap.log python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_project_scenes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "c3 or c5 or deep or normalmap or wide or sort" || exit 99
grep -q " passed" gpurun_out/pytest_shade_nmap.log && ! grep -q " failed" gpurun_out/pytest_shade_nmap.log || { tail -30 gpurun_out/pytest_shade_nmap.log; exit 98; }
grep -E "passed|failed" gpurun_out/pytest_shade_nmap.log | tail -1
for cfg in c3 c5 bumpy1m; do
  bash scripts/ab_libs2.sh 2 "lib_prev lib" --config $cfg --no-extras --strong-spp 0 | sed "s/^/$cfg /" || exit 99
done

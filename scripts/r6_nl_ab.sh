#!/usr/bin/env bash
# round 6: machine-LICM-off build (lib_nl) + persistent bounce grid -- parity subset, then interleaved C2 A/B
set -u
NL=$PWD/optix-renderer_amd/lib_nl/libnori_hip.so
K="c2_full or cbox or variants or tail or textures or normalmap_cbox or multi_chunk or async"
NH_LIB_PATH=$NL scripts/gpu_step.sh 500 gpurun_out/pytest_nl.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -k "$K" || exit 99
tail -2 gpurun_out/pytest_nl.log
grep -q " passed" gpurun_out/pytest_nl.log && ! grep -q " failed" gpurun_out/pytest_nl.log || exit 98
scripts/gpu_step.sh 300 gpurun_out/pytest_r6g.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -k "normalmap or normals" || exit 99
tail -2 gpurun_out/pytest_r6g.log
bash scripts/ab_libs2.sh 2 "lib lib_wa lib_nl" --config c2 --strong-spp 0 --no-extras > gpurun_out/ab_nl_c2.txt 2>&1; cat gpurun_out/ab_nl_c2.txt
NH_LIB_PATH=$NL scripts/ab_env.sh 2 c2 "NH_BOUNCE_PERSIST=0 NH_BOUNCE_PERSIST=4 NH_BOUNCE_PERSIST=2" --no-extras --strong-spp 0 > gpurun_out/ab_nl_persist_c2.txt 2>&1; cat gpurun_out/ab_nl_persist_c2.txt

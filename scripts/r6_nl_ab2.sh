#!/usr/bin/env bash
# round 6: machine-LICM-off builds on every config (lib = default flags, lib_nl = -mllvm -disable-machine-licm,
# lib_nl6 = lib_nl + any-hit persistent traversal at 6 waves/SIMD) -- parity on lib_nl6, then interleaved A/B
set -u
NL=$PWD/optix-renderer_amd/lib_nl6/libnori_hip.so
[ -n "${SKIP_TESTS:-}" ] || NH_LIB_PATH=$NL scripts/gpu_step.sh 900 gpurun_out/pytest_nl6.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread || exit 99
[ -n "${SKIP_TESTS:-}" ] || tail -2 gpurun_out/pytest_nl6.log
[ -n "${SKIP_TESTS:-}" ] || grep -q " passed" gpurun_out/pytest_nl6.log && ! grep -q " failed" gpurun_out/pytest_nl6.log || exit 98
for cfg in ${CFGS:-c3 bumpy1m c5}; do
  bash scripts/ab_libs2.sh 2 "lib lib_nl lib_nl6" --config $cfg --strong-spp 0 --no-extras > gpurun_out/ab_nl_$cfg.txt 2>&1; cat gpurun_out/ab_nl_$cfg.txt
done

#!/usr/bin/env bash
# One A/B session: the GPU suite on the working build, interleaved bench A/B of library builds, and a VALU / wait
# PMC pass per build on one configuration.
# usage: scripts/gpu_ab_session.sh TAG ROUNDS "lib lib_x ..." CONFIG [pytest -k expr | -]
set -u
tag=$1; n=$2; libs=$3; cfg=$4; k=${5:-}
mkdir -p gpurun_out
if [ "$k" != "-" ]; then
  if [ -n "$k" ]; then
    scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -k "$k" || exit 99
  else
    scripts/gpu_step.sh 600 gpurun_out/pytest_$tag.log python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread || exit 99
  fi
  tail -2 gpurun_out/pytest_$tag.log
  grep -q " passed" gpurun_out/pytest_$tag.log && ! grep -q " failed" gpurun_out/pytest_$tag.log || { grep -E "FAIL|Error" gpurun_out/pytest_$tag.log | head -20; exit 98; }
fi
bash scripts/ab_libs2.sh $n "$libs" --config $cfg --strong-spp 0 --no-extras > gpurun_out/ab_$tag.txt 2>&1 || { cat gpurun_out/ab_$tag.txt; exit 99; }
cat gpurun_out/ab_$tag.txt
for v in $libs; do
  if [ $v = lib ]; then unset NH_LIB_PATH; else export NH_LIB_PATH=$PWD/optix-renderer_amd/$v/libnori_hip.so; fi
  scripts/pmc_groups.sh ${tag}_$v "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" -- --config $cfg --strong-spp 0 --no-extras > /dev/null || exit 99
  grep -E "bounce_rr|splat|merge" gpurun_out/pmc_${tag}_$v/summary.txt | grep -E "INSTS_VALU|WAVE_CYCLES|WAIT_ANY|INSTS_LDS" | sed "s/^/$v /"
done

# round 4: the GPU suite and smoke on the final build
set -u
mkdir -p gpurun_out
scripts/gpu_step.sh 150 gpurun_out/smoke_r4final.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
scripts/gpu_step.sh 600 gpurun_out/pytest_r4final.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 99
tail -1 gpurun_out/pytest_r4final.log; cat gpurun_out/smoke_r4final.log

# round 4, first GPU session: r2-vs-HEAD perf-1M A/B, texture parity, per-bounce profile of perf-1M
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_r2_head_1m.sh 3 > gpurun_out/ab1m.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/ab1m.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_textures.py > gpurun_out/pytest_tex.log 2>&1; echo "tex rc=$?"; tail -25 gpurun_out/pytest_tex.log
NH_POOLS=1 NH_TRACE_COUNTS=1 timeout -k 10 300 python bench.py --config bumpy1m --steps 2 --warmup 1 --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 --roofline-steps 0 > gpurun_out/trace1m.log 2>&1; echo "trace rc=$?"; grep "chunk seq" gpurun_out/trace1m.log | tail -3
bash scripts/valu_issue.sh > gpurun_out/valu_issue.txt 2>&1; echo "valu rc=$?"; tail -25 gpurun_out/valu_issue.txt

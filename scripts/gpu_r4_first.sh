# round 4, first GPU session: perf-1M A/B (round 2, round 3, working tree with / without the one-launch trace),
# texture parity, per-bounce profile of perf-1M, VALU issue ceiling
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_r2_head_1m.sh 2 "r2 head cur cur:NH_TRACE2=0" > gpurun_out/ab1m.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/ab1m.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_textures.py > gpurun_out/pytest_tex.log 2>&1; echo "tex rc=$?"; tail -25 gpurun_out/pytest_tex.log
for t in 1 0; do NH_TRACE2=$t NH_POOLS=1 NH_TRACE_COUNTS=1 timeout -k 10 300 python bench.py --config bumpy1m --steps 2 --warmup 1 --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 --roofline-steps 0 > gpurun_out/trace1m_$t.log 2>&1; echo "trace$t rc=$?"; grep "chunk seq" gpurun_out/trace1m_$t.log | tail -2; done
bash scripts/valu_issue.sh > gpurun_out/valu_issue.txt 2>&1; echo "valu rc=$?"; tail -25 gpurun_out/valu_issue.txt
for cfg in c1 c4; do timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu --no-denoise --no-extras --strong-spp 0 --traversal-1m-steps 0 > gpurun_out/tailprof_$cfg.log 2>&1; echo "tailprof $cfg rc=$?"; python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/tailprof_$cfg.log') if x.startswith('{')][0]); r=d['roofline']
print('$cfg', d['value'], r.get('tail_profile'), {k: (v['ms'], v['launches']) for k, v in r['stages'].items()})"; done

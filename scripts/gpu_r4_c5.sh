# round 4: C5 with the split traversal launches again (tree past the MALL), C3 and perf-1M with the fused one
set -o pipefail
mkdir -p gpurun_out
for cfg in c5 c3 bumpy1m; do
  steps=4; [ $cfg = c5 ] && steps=3; [ $cfg = c3 ] && steps=2
  scripts/gpu_step.sh 300 gpurun_out/bench_r4g_$cfg.log python bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-denoise --traversal-1m-steps 0 --strong-spp 0 --no-extras || exit 99
done
grep -h '^{' gpurun_out/bench_r4g_*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['config'], json.loads(l)['value'], json.loads(l)['config'].get('trace_fused')) for l in sys.stdin]"

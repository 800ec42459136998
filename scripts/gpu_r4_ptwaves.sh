# round 4: waves per SIMD of the persistent traversal kernels (wf_trace_pt2 on perf-1M): 5 (default) vs 6 / 4 builds
set -o pipefail
mkdir -p gpurun_out
L=NH_LIB_PATH=optix-renderer_amd
bash scripts/ab_variants.sh bumpy1m 2 "cur cur:$L/vW6/libnori_hip.so cur:$L/vW4/libnori_hip.so" > gpurun_out/ab22_1m.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/ab22_1m.txt

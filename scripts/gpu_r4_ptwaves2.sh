# round 4: persistent traversal at 4 waves/SIMD (vW4 build) vs 5 on C3 and C5
set -o pipefail
mkdir -p gpurun_out
L=NH_LIB_PATH=optix-renderer_amd
bash scripts/ab_variants.sh c3 2 "cur cur:$L/vW4/libnori_hip.so" > gpurun_out/ab22_c3.txt 2>&1; echo "ab c3 rc=$?"; cat gpurun_out/ab22_c3.txt
bash scripts/ab_variants.sh c5 1 "cur cur:$L/vW4/libnori_hip.so" > gpurun_out/ab22_c5.txt 2>&1; echo "ab c5 rc=$?"; cat gpurun_out/ab22_c5.txt

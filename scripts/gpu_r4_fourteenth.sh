# round 4, fourteenth GPU session: C2 cost attribution of this round's shading changes -- builds with textures
# (vA), the isolated-sphere test (vB), and those plus the light-sample skip (vC) compiled out, against round 3's HEAD
set -o pipefail
mkdir -p gpurun_out
L=NH_LIB_PATH=optix-renderer_amd
bash scripts/ab_variants.sh c2 3 "head cur cur:$L/vA/libnori_hip.so cur:$L/vB/libnori_hip.so cur:$L/vC/libnori_hip.so" > gpurun_out/ab14_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab14_c2.txt

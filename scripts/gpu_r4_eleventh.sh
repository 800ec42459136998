# round 4, eleventh GPU session: record layout A/B on C2 -- 12-B (r, g, b) records vs 16-B aligned ones
# (optix-renderer_amd/v16: NH_REC_STRIDE=4), jitter recomputed vs stored, against round 3's HEAD
set -o pipefail
mkdir -p gpurun_out
V=NH_LIB_PATH=optix-renderer_amd/v16/libnori_hip.so
bash scripts/ab_variants.sh c2 3 "head cur cur:NH_SPLAT_JITTER=stored cur:$V cur:$V,NH_SPLAT_JITTER=stored" > gpurun_out/ab11_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab11_c2.txt

# round 4: tail threshold with the round-4 tail kernel -- C1 / C4 at the default (64k paths) vs 128k / 256k
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_variants.sh c1 2 "cur cur:NH_TAIL=131072 cur:NH_TAIL=262144" > gpurun_out/ab21_c1.txt 2>&1; echo "ab c1 rc=$?"; cat gpurun_out/ab21_c1.txt
bash scripts/ab_variants.sh c4 2 "cur cur:NH_TAIL=131072 cur:NH_TAIL=262144" > gpurun_out/ab21_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab21_c4.txt

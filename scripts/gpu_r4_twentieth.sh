# round 4, twentieth GPU session: path pools with 8 hardware queues -- C2 at 2 (default) / 3 pools, C4 at 3 (default) / 4
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_variants.sh c2 3 "cur cur:NH_POOLS=3" > gpurun_out/ab20_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab20_c2.txt
bash scripts/ab_variants.sh c4 2 "cur cur:NH_POOLS=4" > gpurun_out/ab20_c4.txt 2>&1; echo "ab c4 rc=$?"; cat gpurun_out/ab20_c4.txt

# round 4, twelfth GPU session: where C2 lost ~2 % against round 3's HEAD in the timed run -- tail register
# budget (NH_TAIL_RR_WAVES=4), lead splat workgroups (NH_SPLAT_LEAD=0), hardware queues (--hw-queues 4)
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_variants.sh c2 3 "head cur cur:NH_TAIL_RR_WAVES=4 cur:NH_SPLAT_LEAD=0" > gpurun_out/ab12_c2.txt 2>&1; echo "ab c2 rc=$?"; cat gpurun_out/ab12_c2.txt
bash scripts/ab_variants.sh c2 3 "cur" --hw-queues 4 > gpurun_out/ab12_c2_q4.txt 2>&1; echo "ab c2 q4 rc=$?"; cat gpurun_out/ab12_c2_q4.txt

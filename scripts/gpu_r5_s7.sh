set -u
mkdir -p gpurun_out
bash scripts/ab_env.sh 2 "c2" "NH_TAIL=65536 NH_TAIL=32768 NH_TAIL=16384 NH_TAIL=8192" --strong-spp 0 --no-extras || exit 99
bash scripts/ab_env.sh 1 "c1 c4" "NH_TAIL=65536 NH_TAIL=32768 NH_TAIL=16384" --strong-spp 0 --no-extras || exit 99

# round 4, thirteenth GPU session: instruction-fetch counters of the C2 bounce kernel (is its ~160 KB of code
# instruction-cache bound?)
set -o pipefail
mkdir -p gpurun_out
bash scripts/pmc_icache.sh c2 --config c2

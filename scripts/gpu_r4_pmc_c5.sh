# round 4 PMC passes for C5's wf_trace_pt2 (10M triangles + envmap: the out-of-cache traversal), one pool
set -o pipefail
mkdir -p gpurun_out
PMC_PASSES="1 4 5 6 7" bash scripts/pmc_valu.sh r4c5 --config c5 --steps 1 --warmup 0 --strong-spp 0 --no-extras || exit 99

#!/usr/bin/env bash
# Full GPU parity suite + smoke + default bench line + rocprofv3 kernel trace + PMC, for one tag.
set -u
tag=$1; shift
mkdir -p gpurun_out
scripts/gpu_step.sh 120 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
grep -q "rel-L2" gpurun_out/smoke_$tag.log || { cat gpurun_out/smoke_$tag.log; exit 98; }
scripts/round_profile.sh "$tag" "$@"

#!/usr/bin/env bash
# PMC passes for one bench configuration, one rocprofv3 --pmc run per counter group (kernel-trace only).
# usage: scripts/pmc_groups.sh TAG "grp1 counters" "grp2 counters" ... -- bench-args...
set -u
tag=$1; shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu --no-calibrate --traversal-1m-steps 0 --roofline-steps 0 --steps 2 --warmup 0 "$@" > $out/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $out/p$i.log; exit 99; }
done
python3 scripts/pmc_summary.py $out > $out/summary.txt && cat $out/summary.txt

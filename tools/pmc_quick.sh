#!/bin/bash
# One rocprofv3 PMC pass over tools/launch_breakdown.py (one-stream c2 batch) per environment
# setting, summarised per recon kernel:  tools/pmc_quick.sh <tag> "<counters>" "ENV=a" "ENV=b" ...
set -u
TAG=$1; CTRS=$2; shift 2
export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  OUT=gpurun_out/pmcq_${TAG}_$i
  mkdir -p $OUT
  env $e timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/p -o p -- python3 tools/launch_breakdown.py --reps 3 > $OUT/p.log 2>&1
  echo "== $e rc=$?"
  python3 tools/counters_summary.py $OUT
done

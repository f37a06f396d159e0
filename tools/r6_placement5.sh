#!/bin/bash
# Round-6 placement probe 5 (gpurun, one box): 6 c2 contexts (tools/placement.py, timed in creation
# order then reversed) with each given option set, one process per set ("-" = none)
set -o pipefail
mkdir -p gpurun_out
n=0
for opts in "$@"; do
  n=$((n+1)); [ "$opts" = "-" ] && opts=""
  timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 6 --steps 10 --reps 2 --no-probe ${opts//,/ } > gpurun_out/placement5_$n.txt 2>&1 || { tail -5 gpurun_out/placement5_$n.txt; exit 1; }
  echo "== $opts"; grep -v '^{' gpurun_out/placement5_$n.txt | sed 's/ per-mode.*//'
done
echo ALL_DONE

#!/bin/bash
# Round-6 placement probe 4 (gpurun, one box): 6 c2 contexts (tools/placement.py) behind a held
# device-memory ballast of each given size (GB), one process per size
set -o pipefail
mkdir -p gpurun_out
for gb in "$@"; do
  timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 6 --steps 10 --reps 1 --no-probe --ballast-gb $gb > gpurun_out/placement4_$gb.txt 2>&1 || { tail -5 gpurun_out/placement4_$gb.txt; exit 1; }
  echo "== ballast $gb GB"; grep -v '^{' gpurun_out/placement4_$gb.txt
done
echo ALL_DONE

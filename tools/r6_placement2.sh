#!/bin/bash
# Round-6 placement probe 2 (gpurun, one box): 6 c2 contexts held at once, each timed round-robin
# twice, then each pool block's HBM rate (tools/placement.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/placement.py --config c2 --contexts 6 --steps 10 --reps 2 > gpurun_out/placement2_2s.txt 2>&1 || exit 1
grep -v '^{' gpurun_out/placement2_2s.txt
echo ALL_DONE

#!/bin/bash
# Round-6 placement probe (gpurun, one box): 4 c2 contexts held at once, two-stream then one-stream,
# each timed round-robin twice (tools/placement.py), then the default c2 bench line twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 4 --steps 10 --reps 2 > gpurun_out/placement_2s.txt 2>&1 || exit 1
cat gpurun_out/placement_2s.txt
timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 4 --steps 6 --reps 2 --one-stream > gpurun_out/placement_1s.txt 2>&1 || exit 1
cat gpurun_out/placement_1s.txt
ROUNDS=1 bash tools/ab5.sh 2 base > gpurun_out/ab_r6i.txt || exit 1
cat gpurun_out/ab_r6i.txt
echo ALL_DONE

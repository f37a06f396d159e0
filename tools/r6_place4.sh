#!/bin/bash
# Round-6: c2 bench A/B, placement calibration on (default) vs off, with the per-kernel context
# allocated before the calibration; 3 interleaved rounds
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_PLACE_CANDIDATES=1 > gpurun_out/ab_r6_place4.txt || { cat gpurun_out/ab_r6_place4.txt; exit 1; }
cat gpurun_out/ab_r6_place4.txt
echo ALL_DONE

#!/bin/bash
# Round-6: c2 bench, placement calibration with the discarded pools freed (default) or held
# (MP2VG_PLACE_HOLD=1), against no calibration; 3 interleaved rounds
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_PLACE_HOLD=1 base@MP2VG_PLACE_CANDIDATES=1 > gpurun_out/ab_r6_place_hold.txt || { cat gpurun_out/ab_r6_place_hold.txt; exit 1; }
cat gpurun_out/ab_r6_place_hold.txt
echo ALL_DONE

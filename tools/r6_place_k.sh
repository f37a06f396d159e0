#!/bin/bash
# Round-6: placement calibration with 4 candidate pools (new default) against 3, c2, 4 interleaved
# rounds (each process its own placements); then c3 once (memory guards)
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 4 base base@MP2VG_PLACE_CANDIDATES=3 > gpurun_out/ab_r6_place_k.txt || { cat gpurun_out/ab_r6_place_k.txt; exit 1; }
cat gpurun_out/ab_r6_place_k.txt
CFG=c3 ROUNDS=1 bash tools/ab5.sh 1 base > gpurun_out/ab_r6_place_k_c3.txt || { cat gpurun_out/ab_r6_place_k_c3.txt; exit 1; }
cat gpurun_out/ab_r6_place_k_c3.txt
echo ALL_DONE

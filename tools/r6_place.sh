#!/bin/bash
# Round-6: c2 bench A/B of the pool placement calibration (MP2VG_PLACE_CANDIDATES pools tried at
# the first batch, the fastest kept; one-stream contexts too with MP2VG_PLACE_ONE_STREAM=1),
# 3 interleaved rounds, then the calibration's own trace lines
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_PLACE_CANDIDATES=3,MP2VG_TRACE=1 base@MP2VG_PLACE_CANDIDATES=3,MP2VG_PLACE_ONE_STREAM=1 > gpurun_out/ab_r6_place.txt || { cat gpurun_out/ab_r6_place.txt; exit 1; }
cat gpurun_out/ab_r6_place.txt
grep -h "placement:" gpurun_out/ab5/c2_base_MP2VG_PLACE_CANDIDATES_3_MP2VG_TRACE_1.*.err
echo ALL_DONE

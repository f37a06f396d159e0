#!/bin/bash
# Round-6: GPU tests with the placement calibration on by default, then the c2 bench A/B against
# it turned off (MP2VG_PLACE_CANDIDATES=1), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_place.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_place.log; [ $rc = 0 ] || exit 1
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_PLACE_CANDIDATES=1 > gpurun_out/ab_r6_place3.txt || { cat gpurun_out/ab_r6_place3.txt; exit 1; }
cat gpurun_out/ab_r6_place3.txt
echo ALL_DONE

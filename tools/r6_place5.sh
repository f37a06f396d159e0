#!/bin/bash
# Round-6: c2 bench, placement calibration on/off x per-kernel context allocated late (default) /
# early (MP2VG_BENCH_CTX1_EARLY=1), 2 interleaved rounds on one box
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 2 base base@MP2VG_PLACE_CANDIDATES=1 base@MP2VG_BENCH_CTX1_EARLY=1 base@MP2VG_BENCH_CTX1_EARLY=1,MP2VG_PLACE_CANDIDATES=1 > gpurun_out/ab_r6_place5.txt || { cat gpurun_out/ab_r6_place5.txt; exit 1; }
cat gpurun_out/ab_r6_place5.txt
echo ALL_DONE

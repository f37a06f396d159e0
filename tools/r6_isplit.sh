#!/bin/bash
# Round-6: I launches in pieces of a row (dev MP2VG_I_SPLIT): c1, c5 and c2 A/B, interleaved
set -o pipefail
CFG=c1 ROUNDS=1 bash tools/ab5.sh 3 dev dev@MP2VG_I_SPLIT=2 dev@MP2VG_I_SPLIT=3 > gpurun_out/ab_r6_isplit_c1.txt || { cat gpurun_out/ab_r6_isplit_c1.txt; exit 1; }
cat gpurun_out/ab_r6_isplit_c1.txt
CFG=c5 ROUNDS=1 bash tools/ab5.sh 2 dev dev@MP2VG_SLICE_ROWS_I=1 dev@MP2VG_SLICE_ROWS_I=1,MP2VG_I_SPLIT=2 > gpurun_out/ab_r6_isplit_c5.txt || { cat gpurun_out/ab_r6_isplit_c5.txt; exit 1; }
cat gpurun_out/ab_r6_isplit_c5.txt
CFG=c2 ROUNDS=1 bash tools/ab5.sh 2 dev dev@MP2VG_I_SPLIT=2 > gpurun_out/ab_r6_isplit_c2.txt || { cat gpurun_out/ab_r6_isplit_c2.txt; exit 1; }
cat gpurun_out/ab_r6_isplit_c2.txt
echo ALL_DONE

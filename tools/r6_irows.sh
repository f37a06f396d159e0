#!/bin/bash
# Round-6: I-launch slices of 2 or 4 MB rows (dev MP2VG_SLICE_ROWS_I) against one row: c1 and c2
set -o pipefail
CFG=c1 ROUNDS=1 bash tools/ab5.sh 3 dev dev@MP2VG_SLICE_ROWS_I=2 dev@MP2VG_SLICE_ROWS_I=4 > gpurun_out/ab_r6_irows_c1.txt || { cat gpurun_out/ab_r6_irows_c1.txt; exit 1; }
cat gpurun_out/ab_r6_irows_c1.txt
CFG=c2 ROUNDS=1 bash tools/ab5.sh 2 dev dev@MP2VG_SLICE_ROWS_I=2 > gpurun_out/ab_r6_irows_c2.txt || { cat gpurun_out/ab_r6_irows_c2.txt; exit 1; }
cat gpurun_out/ab_r6_irows_c2.txt
echo ALL_DONE

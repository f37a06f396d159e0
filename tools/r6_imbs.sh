#!/bin/bash
# Round-6: I slices of N MBs cut across rows (dev MP2VG_I_SLICE_MBS): whole rounds of resident
# workgroups; c5 (4:4:4, 2-row slices = 240 MBs) and c1 (1 row = 120 MBs)
set -o pipefail
CFG=c5 ROUNDS=1 bash tools/ab5.sh 3 dev dev@MP2VG_I_SLICE_MBS=256 dev@MP2VG_I_SLICE_MBS=252 > gpurun_out/ab_r6_imbs_c5.txt || { cat gpurun_out/ab_r6_imbs_c5.txt; exit 1; }
cat gpurun_out/ab_r6_imbs_c5.txt
CFG=c1 ROUNDS=1 bash tools/ab5.sh 3 dev dev@MP2VG_I_SLICE_MBS=128 dev@MP2VG_I_SLICE_MBS=160 > gpurun_out/ab_r6_imbs_c1.txt || { cat gpurun_out/ab_r6_imbs_c1.txt; exit 1; }
cat gpurun_out/ab_r6_imbs_c1.txt
echo ALL_DONE

#!/bin/bash
# Round-6: intra dequant DC select as sbfe + bfi (variant exec: dead lanes of the last word round masked by exec, not by address) against the default, c5 and c1,
# 3 interleaved rounds each (bench line and the calibrated one-stream I launch)
set -o pipefail
CFG=c5 ROUNDS=1 bash tools/ab5.sh 3 base exec > gpurun_out/ab_r6_exec_c5.txt || { cat gpurun_out/ab_r6_exec_c5.txt; exit 1; }
cat gpurun_out/ab_r6_exec_c5.txt
CFG=c1 ROUNDS=1 bash tools/ab5.sh 3 base exec > gpurun_out/ab_r6_exec_c1.txt || { cat gpurun_out/ab_r6_exec_c1.txt; exit 1; }
cat gpurun_out/ab_r6_exec_c1.txt
echo ALL_DONE

#!/bin/bash
# Round-6: intra dequant DC select as sbfe + bfi (variant kb8: k*8 in the kbtab entry low bits) against the default, c5 and c1,
# 3 interleaved rounds each (bench line and the calibrated one-stream I launch)
set -o pipefail
CFG=c5 ROUNDS=1 bash tools/ab5.sh 3 base kb8 > gpurun_out/ab_r6_kb8_c5.txt || { cat gpurun_out/ab_r6_kb8_c5.txt; exit 1; }
cat gpurun_out/ab_r6_kb8_c5.txt
CFG=c1 ROUNDS=1 bash tools/ab5.sh 3 base kb8 > gpurun_out/ab_r6_kb8_c1.txt || { cat gpurun_out/ab_r6_kb8_c1.txt; exit 1; }
cat gpurun_out/ab_r6_kb8_c1.txt
echo ALL_DONE

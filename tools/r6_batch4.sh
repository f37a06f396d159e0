#!/bin/bash
# Round-6 batch 4 (gpurun, one box): evidence of the built library (GPU tests, smoke, bench lines
# c1-c5, tools/r6_evidence.sh), then the c1 A/B of the mode-4 I launch (dev library, 3 rounds)
set -o pipefail
bash tools/r6_evidence.sh ${1:-a} || exit 1
CFG=c1 bash tools/ab5.sh 3 dev dev@MP2VG_I_TILEFREE=0 > gpurun_out/ab_r6_mode4_c1.txt || { cat gpurun_out/ab_r6_mode4_c1.txt; exit 1; }
cat gpurun_out/ab_r6_mode4_c1.txt
echo ALL_DONE

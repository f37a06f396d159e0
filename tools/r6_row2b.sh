#!/bin/bash
# Round-6: the B loop's row-2 loads (variant r2, MP2VG_ROW2_LOAD=1) against the default, now that
# each process calibrates its pool placement; 3 interleaved rounds, c2
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base r2 > gpurun_out/ab_r6_row2_calibrated.txt || { cat gpurun_out/ab_r6_row2_calibrated.txt; exit 1; }
cat gpurun_out/ab_r6_row2_calibrated.txt
echo ALL_DONE

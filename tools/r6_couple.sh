#!/bin/bash
# Round-6: coupling of the two picture sets' launch chains (dev MP2VG_SET_COUPLE: 0 free-running
# = default, 1 lockstep, 2 staggered), c2, 2 interleaved rounds
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 2 dev dev@MP2VG_SET_COUPLE=1 dev@MP2VG_SET_COUPLE=2 > gpurun_out/ab_r6_couple.txt || { cat gpurun_out/ab_r6_couple.txt; exit 1; }
cat gpurun_out/ab_r6_couple.txt
echo ALL_DONE

#!/bin/bash
# Round-6: c2 picture sets per batch (MP2VG_STREAMS 2 = default, 3, 4), 3 interleaved rounds
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_STREAMS=3 base@MP2VG_STREAMS=4 > gpurun_out/ab_r6_streams.txt || { cat gpurun_out/ab_r6_streams.txt; exit 1; }
cat gpurun_out/ab_r6_streams.txt
echo ALL_DONE

#!/bin/bash
# Round-6: c2 bench A/B of the dev library with helper streams taking the first hardware queues
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 dev dev@MP2VG_QUEUE_WARM=2 dev@MP2VG_QUEUE_WARM=4 > gpurun_out/ab_r6q.txt || { cat gpurun_out/ab_r6q.txt; exit 1; }
cat gpurun_out/ab_r6q.txt
echo ALL_DONE

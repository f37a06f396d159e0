#!/bin/bash
# Round-6: LLVM AMDGPU scheduler strategies (variants s_max-ilp, s_max-memory-clause) against the
# default, c2 bench, 2 interleaved rounds
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 2 base s_max-ilp s_max-memory-clause > gpurun_out/ab_r6_sched.txt || { cat gpurun_out/ab_r6_sched.txt; exit 1; }
cat gpurun_out/ab_r6_sched.txt
echo ALL_DONE

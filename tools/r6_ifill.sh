#!/bin/bash
# Round-6: I slices sized to fill whole rounds (new default) against the row slices (dev
# MP2VG_SLICE_ROWS_I=1, or 2 for 4:4:4): GPU tests, then c1 / c5 / c2 A/B, interleaved
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ifill.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_ifill.log; [ $rc = 0 ] || exit 1
CFG=c1 ROUNDS=1 bash tools/ab5.sh 4 dev dev@MP2VG_SLICE_ROWS_I=1 > gpurun_out/ab_r6_ifill_c1.txt || { cat gpurun_out/ab_r6_ifill_c1.txt; exit 1; }
cat gpurun_out/ab_r6_ifill_c1.txt
CFG=c5 ROUNDS=1 bash tools/ab5.sh 4 dev dev@MP2VG_SLICE_ROWS_I=2 > gpurun_out/ab_r6_ifill_c5.txt || { cat gpurun_out/ab_r6_ifill_c5.txt; exit 1; }
cat gpurun_out/ab_r6_ifill_c5.txt
CFG=c2 ROUNDS=1 bash tools/ab5.sh 2 dev dev@MP2VG_SLICE_ROWS_I=1 > gpurun_out/ab_r6_ifill_c2.txt || { cat gpurun_out/ab_r6_ifill_c2.txt; exit 1; }
cat gpurun_out/ab_r6_ifill_c2.txt
echo ALL_DONE

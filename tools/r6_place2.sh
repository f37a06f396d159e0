#!/bin/bash
# Round-6: placement calibration seen from tools/placement.py: 3 contexts, calibrated at their
# first batch (MP2VG_PLACE_CANDIDATES=3, trace on), then timed round-robin, two-stream and one-stream
set -o pipefail
for os in "" "--one-stream"; do
  MP2VG_PLACE_CANDIDATES=3 MP2VG_TRACE=1 timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 3 --steps 10 --reps 2 --no-probe $os > gpurun_out/place2$os.txt 2>&1 || { tail -5 gpurun_out/place2$os.txt; exit 1; }
  echo "== $os"; grep -E "placement:|ms/batch" gpurun_out/place2$os.txt | sed 's/ per-mode.*//'
done
echo ALL_DONE

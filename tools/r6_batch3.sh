#!/bin/bash
# Round-6 batch 3 (gpurun, one box): c2 A/B of the tap-issue changes with a one-stream arm (box
# spread attribution), the drop-in frame modes, the intra dequant table on c1/c5/c2, and the I-only
# configs at 4x their frame counts
set -o pipefail
AB='base head r2only base@MP2VG_STREAMS=1' ROUNDS=2 CFG=c2 bash tools/stamps_ab.sh r6g || exit 1
cat gpurun_out/ab_r6g.txt
bash tools/r6_dropin.sh || exit 1
bash tools/r6_batch2.sh || exit 1
echo ALL_DONE

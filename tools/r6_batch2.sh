#!/bin/bash
# Round-6 batch 2 (gpurun): the intra dequant's (MB, block) table on the I-only configs and c2,
# then the I-only configs at 4x their round-5 frame counts
set -o pipefail
mkdir -p gpurun_out
for cfg in c1 c5; do
  CFG=$cfg timeout -k 10 900 tools/ab5.sh 3 base nokb > gpurun_out/ab_r6h_$cfg.txt 2>&1 || { cat gpurun_out/ab_r6h_$cfg.txt; exit 1; }
  cat gpurun_out/ab_r6h_$cfg.txt
done
bash tools/r6_batchsize.sh

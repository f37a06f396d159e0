#!/bin/bash
# Round-6 batch 1 (gpurun): tile-free I launches forced (dev), chroma taps from frame rows
# (variant ct0: no chroma tiles), FETCH/WRITE of ct0 and base on the one-stream batch
set -o pipefail
mkdir -p gpurun_out
CFG=c2 timeout -k 10 900 tools/ab5.sh 2 dev dev@MP2VG_I_TILEFREE=2 base ct0 > gpurun_out/ab_r6c.txt 2>&1 || exit 1
for v in base ct0; do
  L=""; [ $v != base ] && L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so
  MP2VG_LIB=$L PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" CFG=c2 REPS=2 timeout -k 10 600 bash tools/pmc5.sh r6c_$v > gpurun_out/pmc5_r6c_$v.txt 2>&1 || exit 1
done
echo done

#!/bin/bash
# pool placement study: per-pool step times (tools/pool_var.py) under slot pads and allocation modes
#   PADS="0 4352" ALLOCS="0 1" CFGS="c3 c2" tools/r4_pad.sh
set -o pipefail
mkdir -p gpurun_out/r4pad
for c in ${CFGS:-c3}; do
  for a in ${ALLOCS:-0 1}; do
    for pad in ${PADS:-0 256 4352 65792}; do
      MP2VG_POOL_ALLOC=$a MP2VG_SLOT_PAD=$pad MP2VG_TILE_PAD=${TPAD:-$pad} timeout -k 10 240 python -u tools/pool_var.py $c ${TRIALS:-2} > gpurun_out/r4pad/$c.a$a.p$pad.log 2>&1 || { tail -5 gpurun_out/r4pad/$c.a$a.p$pad.log; exit 1; }
      echo "$c alloc=$a pad=$pad: $(grep -o '[0-9.]* ms/step' gpurun_out/r4pad/$c.a$a.p$pad.log | awk '{print $1}' | tr '\n' ' ')"
    done
  done
done

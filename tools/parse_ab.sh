#!/bin/bash
# host parse rate of the in-tree library vs a variant library (1 and 16 threads, interleaved)
#   tools/parse_ab.sh <variant> <rounds>
V=$1; R=${2:-2}
for r in $(seq 1 $R); do
  for L in "" tiny_mp2v_dec_amd/_var/$V/libmp2vg.so; do
    echo "${L:-in-tree}: $(MP2VG_LIB=$L timeout -k 10 120 python tools/parse_scale.py | tr '\n' ' ')" || exit 1
  done
done

#!/bin/bash
# drop-in end-to-end A/B of the in-tree library against variant libraries (interleaved rounds):
#   tools/e2e_ab.sh <rounds> <variant>...      (c2 bench stream, 64 GOPs, 16 host threads)
R=$1; shift
for r in $(seq 1 $R); do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
    echo "$v $(MP2VG_LIB=$L timeout -k 10 200 python tools/e2e_bench.py --gops 64 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["dropin_fps"])')" || exit 1
  done
done

#!/bin/bash
# drop-in phase breakdown (MP2VG_TRACE) of the in-tree library and variants, interleaved:
#   tools/e2e_trace_ab.sh <rounds> <variant>...
R=$1; shift
for r in $(seq 1 $R); do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
    MP2VG_TRACE=1 MP2VG_LIB=$L timeout -k 10 200 python tools/e2e_bench.py --gops 64 > gpurun_out/tr_$v.log 2>&1 || exit 1
    echo "$v $(grep -E "dropin: (headers|parse wait|gather|upload|decode issue|download wait|after parse)" gpurun_out/tr_$v.log | awk '{printf "%s=%s ", $3, $(NF-1)}') fps=$(tail -1 gpurun_out/tr_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["dropin_fps"])')"
  done
done

#!/bin/bash
# drop-in phase breakdown (MP2VG_TRACE) under environment settings, interleaved:
#   tools/e2e_trace_env.sh <rounds> "" "VAR=value" ...      ("" = no extra setting)
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    env MP2VG_TRACE=1 $kv timeout -k 10 200 python tools/e2e_bench.py --gops 64 > gpurun_out/tre_$i.log 2>&1 || exit 1
    echo "[${kv:-base}] $(grep -E "dropin: (headers|parse wait|gather|upload|decode issue|download wait|after parse)" gpurun_out/tre_$i.log | awk '{printf "%s=%s ", $3, $(NF-1)}') fps=$(tail -1 gpurun_out/tre_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["dropin_fps"])')"
  done
done

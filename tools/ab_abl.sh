#!/bin/bash
# timing-only A/B of ablation variants (wrong output: bench.py exits 3 on the parity mismatch,
# which is expected here)
#   tools/ab_abl.sh "<bench args>" <rounds> <variant>...
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
    MP2VG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
    rc=$?; [ $rc = 0 -o $rc = 3 ] || { tail -5 gpurun_out/ab/$v.err; exit 1; }
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/$v.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['parity']['status'])")"
  done
done

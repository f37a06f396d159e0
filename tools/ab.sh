#!/bin/bash
# interleaved A/B of the default build vs variants: tools/ab.sh <rounds> <variant>...
R=$1; shift
for r in $(seq 1 $R); do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
    MP2VG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --gops 32 --steps 10 > gpurun_out/ab_$v.log 2>&1 || exit 1
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['kernel_ms_per_step'], d['frame_digest_of_digests'])")"
  done
done

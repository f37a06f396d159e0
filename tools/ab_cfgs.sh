#!/bin/bash
# interleaved A/B of the in-tree build against variant libraries over several configs:
#   tools/ab_cfgs.sh <rounds> "<configs>" <variant>...   (prints value, ms/step, frac, parity per run)
R=$1; CFGS=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for c in $CFGS; do
    for v in base "$@"; do
      if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
      MP2VG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --config $c > gpurun_out/ab/$v.$c.json 2> gpurun_out/ab/$v.$c.err || { tail -5 gpurun_out/ab/$v.$c.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.loads(open('gpurun_out/ab/$v.$c.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'])")"
    done
  done
done

#!/bin/bash
# timing-only A/B of dev variants under one MP2VG_ABLATE value (wrong output: bench.py exits 3
# on the parity mismatch, expected here), interleaved over rounds, per-kernel means printed
#   tools/ab_env_abl.sh <ablate> "<bench args>" <rounds> <variant>...
ABL=$1; ARGS=$2; R=$3; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in "$@"; do
    MP2VG_ABLATE=$ABL MP2VG_LIB=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-e2e $ARGS > gpurun_out/ab/$v.$r.json 2> gpurun_out/ab/$v.$r.err
    rc=$?; [ $rc = 0 -o $rc = 3 ] || { tail -5 gpurun_out/ab/$v.$r.err; exit 1; }
    echo "$v r$r $(python3 -c "
import json;d=json.loads(open('gpurun_out/ab/$v.$r.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel'];print(d['value'], d['ms_per_step'], ' '.join(f\"{k[-8:]}:{v['avg_launch_ms']}\" for k,v in pk.items()))")"
  done
done

#!/bin/bash
# timing-only A/B of MP2VG_ABLATE values on one dev variant library, interleaved over rounds
# (wrong output: bench.py exits 3 on the parity mismatch, expected here)
#   tools/ab_abl_values.sh <variant> "<bench args>" <rounds> <ablate value>...
V=$1; ARGS=$2; R=$3; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for a in "$@"; do
    MP2VG_ABLATE=$a MP2VG_LIB=tiny_mp2v_dec_amd/_var/$V/libmp2vg.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e $ARGS > gpurun_out/ab/$V.$a.$r.json 2> gpurun_out/ab/$V.$a.$r.err
    rc=$?; [ $rc = 0 -o $rc = 3 ] || { tail -5 gpurun_out/ab/$V.$a.$r.err; exit 1; }
    echo "$V abl=$a r$r $(python3 -c "
import json;d=json.loads(open('gpurun_out/ab/$V.$a.$r.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel'];print(d['value'], d['ms_per_step'], ' '.join(f\"{k[-8:-1]}:{v['avg_launch_ms']}\" for k,v in pk.items()))")"
  done
done

#!/bin/bash
# c5 (4:4:4 I-only) timing under dev ablations (variant library tiny_mp2v_dec_amd/_var/abl444, wrong
# output except 0: bench.py exits 3 on the parity mismatch, which is expected here)
for a in 0 1 4 5 8 0; do
  MP2VG_LIB=${MP2VG_LIB:-tiny_mp2v_dec_amd/_var/dev/libmp2vg.so} MP2VG_ABLATE=$a timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-e2e --steps 10 > gpurun_out/c5abl_$a.json 2>gpurun_out/c5abl_$a.err
  rc=$?; [ $rc = 0 -o $rc = 3 ] || { tail -3 gpurun_out/c5abl_$a.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/c5abl_$a.json').read().strip().splitlines()[-1]);print($a, d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'])"
done

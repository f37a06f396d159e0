#!/bin/bash
# interleaved same-box A/B: in-tree library (optionally under env settings) against variant
# libraries, per config, R rounds; prints frames/s, ms/step, frac, parity and per-kernel launch ms
#   tools/ab_cfg_env.sh "<configs>" <rounds> "<bench args>" <arm>...
#   arm = variant name (tiny_mp2v_dec_amd/_var/<name>/libmp2vg.so), "base", or "base:VAR=val,VAR2=val"
CFGS=$1; R=$2; ARGS=$3; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for c in $CFGS; do
    for arm in "$@"; do
      L=""; ENVS=""
      case $arm in
        base) ;;
        base:*) ENVS=$(echo ${arm#base:} | tr ',' ' ') ;;
        *) L=tiny_mp2v_dec_amd/_var/$arm/libmp2vg.so ;;
      esac
      tag=$(echo "$arm" | tr ':=,' '___')
      env $ENVS MP2VG_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --config $c $ARGS > gpurun_out/ab/$tag.$c.$r.json 2> gpurun_out/ab/$tag.$c.$r.err
      rc=$?; [ $rc = 0 ] || { tail -5 gpurun_out/ab/$tag.$c.$r.err; exit 1; }
      echo "$c $arm r$r $(python3 -c "
import json;d=json.loads(open('gpurun_out/ab/$tag.$c.$r.json').read().strip().splitlines()[-1])
pk=d['roofline']['per_kernel'];print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'], ' '.join(f\"{k[-8:-1]}:{v['avg_launch_ms']}\" for k,v in pk.items()))")"
    done
  done
done

#!/bin/bash
# Interleaved bench A/B of the in-tree build against variant libraries (tools/variant.sh), one
# line per run: frames/s, ms/step, frac, parity, one-stream per-kernel launch ms (I / B / P+B ...)
#   CFG=c2 tools/ab5.sh <rounds> <variant>...      (variant "base" = the in-tree library;
#   "name@ENV=VAL" runs library `name` with an environment variable set; exit 3 = parity mismatch, expected
#   for the timing-only MP2VG_ABLATE arms of the dev build)
R=$1; shift
CFG=${CFG:-c2}
mkdir -p gpurun_out/ab5
for r in $(seq 1 $R); do
  for arm in "$@"; do
    v=${arm%%@*}; envs=""; [ "$arm" != "$v" ] && envs=${arm#*@}
    if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
    tag=$(echo "$arm" | tr '=@,' '___')
    env MP2VG_LIB=$L ${envs//,/ } timeout -k 10 240 python bench.py --no-cpu-baseline --no-e2e --config $CFG ${BENCH_ARGS:-} \
      > gpurun_out/ab5/${CFG}_$tag.$r.json 2> gpurun_out/ab5/${CFG}_$tag.$r.err
    rc=$?
    if [ $rc != 0 ] && [ $rc != 3 ]; then echo "$arm rc=$rc"; tail -3 gpurun_out/ab5/${CFG}_$tag.$r.err; exit 1; fi
    python3 - gpurun_out/ab5/${CFG}_$tag.$r.json "$arm" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
pk = " ".join(f"{v['mode']}:{v['avg_launch_ms']}" for v in r["per_kernel"].values())
print(f"{sys.argv[2]:28s} {d['value']:>10.1f} {d['ms_per_step']:7.3f} {r['frac']:.4f} {d['parity']['status']:9s} span1 {r['one_stream_span_ms']:.3f} {pk}", flush=True)
PY
  done
done

#!/bin/bash
# picture-set (stream) count A/B for one bench config, interleaved rounds:
#   tools/ab_streams_cfg.sh <config> <rounds> <nstreams>...
CFG=$1; R=$2; shift 2
mkdir -p gpurun_out/abs
for r in $(seq 1 $R); do
  for n in "$@"; do
    MP2VG_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --config $CFG > gpurun_out/abs/$n.json 2> gpurun_out/abs/$n.err || { tail -5 gpurun_out/abs/$n.err; exit 1; }
    echo "$CFG streams=$n $(python3 -c "import json;d=json.loads(open('gpurun_out/abs/$n.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'])")"
  done
done

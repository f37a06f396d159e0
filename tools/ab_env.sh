#!/bin/bash
# Interleaved A/B of one build under different environment settings:
#   tools/ab_env.sh "<bench args>" <rounds> "ENV=a" "ENV=b" ...
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out/abenv
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/abenv/$i.json 2> gpurun_out/abenv/$i.err || { tail -5 gpurun_out/abenv/$i.err; exit 1; }
    echo "$e $(python3 -c "import json;d=json.loads(open('gpurun_out/abenv/$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'], {k.split('<')[1][:7]: v['avg_launch_ms'] for k, v in d['roofline']['per_kernel'].items()})")"
  done
done

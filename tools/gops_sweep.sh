#!/bin/bash
# c2 throughput vs GOPs per step (batch size), interleaved rounds:  tools/gops_sweep.sh "<gops...>" <rounds> [config]
G=$1; R=${2:-1}; C=${3:-c2}
mkdir -p gpurun_out/gops
for r in $(seq 1 $R); do
  for g in $G; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --config $C --gops $g > gpurun_out/gops/$C.$g.json 2> gpurun_out/gops/$C.$g.err || { tail -5 gpurun_out/gops/$C.$g.err; exit 1; }
    echo "$C gops=$g $(python3 -c "import json;d=json.loads(open('gpurun_out/gops/$C.$g.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'])")"
  done
done

#!/bin/bash
# Round-6: I-only configs at their round-5 batch and at 4x the frames (launch ramps/tails), same box
set -o pipefail
mkdir -p gpurun_out/bs
for r in 1; do
  for arm in "c1 120" "c1 480" "c5 64" "c5 256"; do
    set -- $arm
    timeout -k 10 240 python bench.py --no-cpu-baseline --no-e2e --config $1 --gops $2 --steps 20 > gpurun_out/bs/$1_$2.$r.json 2> gpurun_out/bs/$1_$2.$r.err || { tail -3 gpurun_out/bs/$1_$2.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bs/$1_$2.$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$1 $2', d['value'], d['ms_per_step'], r['frac'], d['parity']['status'], r['one_stream_span_ms'], d['box'])"
  done
done

#!/bin/bash
# Round-6: bench c3 and c4 lines with the final build (per-kernel contexts hold their candidates)
set -o pipefail
mkdir -p gpurun_out/r6_f
for c in c3 c4 c2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e --config $c > gpurun_out/r6_f/bench_$c.json 2> gpurun_out/r6_f/bench_$c.err || { tail -5 gpurun_out/r6_f/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], d['parity']['status'], 'span1', r['one_stream_span_ms'], {k: (v['avg_launch_ms'], v['frac']) for k, v in r['per_kernel'].items()})" gpurun_out/r6_f/bench_$c.json $c
done
echo ALL_DONE

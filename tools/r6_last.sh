#!/bin/bash
# Round-6 last evidence (gpurun): GPU tests, smoke, c1 / c5 bench lines, one-stream rocprof c2
set -o pipefail
mkdir -p gpurun_out/r6_last
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_last/gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6_last/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_last/smoke.log 2>&1 || { tail -5 gpurun_out/r6_last/smoke.log; exit 1; }
tail -1 gpurun_out/r6_last/smoke.log
for c in c1 c5; do
  timeout -k 10 400 python bench.py --no-e2e --config $c > gpurun_out/r6_last/bench_$c.json 2> gpurun_out/r6_last/bench_$c.err || { tail -5 gpurun_out/r6_last/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], d['parity']['status'], 'span1', r['one_stream_span_ms'], {k: (v['avg_launch_ms'], v['frac']) for k, v in r['per_kernel'].items()})" gpurun_out/r6_last/bench_$c.json $c
done
CFG=c2 bash tools/pmc5.sh last_c2 > gpurun_out/r6_last/pmc5_c2.txt 2>&1 || { tail -5 gpurun_out/r6_last/pmc5_c2.txt; exit 1; }
echo ALL_DONE

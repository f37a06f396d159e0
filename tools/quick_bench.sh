#!/bin/bash
# GPU tests, then bench lines of the given configs (no CPU baseline / e2e)
#   tools/quick_bench.sh <tag> <config>...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/$TAG/gpu_tests.log)"
if [ $rc != 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/$TAG/gpu_tests.log | head -20; exit 1; fi
for r in 1 2; do for c in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --config $c --steps 10 > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || { tail -5 gpurun_out/$TAG/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/$TAG/bench_$c.json').read().strip().splitlines()[-1]);print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['status'])"
done; done

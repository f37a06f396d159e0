#!/bin/bash
# GPU tests of the in-tree build, then one bench line per config (no CPU baseline, no e2e)
#   CFGS="c1 c5 c2" tools/r4_quick.sh <tag>
set -o pipefail
OUT=gpurun_out/q_$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit 1; }
for c in ${CFGS:-c1 c5 c2}; do
  timeout -k 10 300 python bench.py --no-e2e --no-cpu-baseline --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1])
r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['frac'],d['parity']['status'],{k[-8:-1]:v['avg_launch_ms'] for k,v in r['per_kernel'].items()})"
done

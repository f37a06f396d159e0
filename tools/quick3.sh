#!/bin/bash
# Quick GPU check of the current build: GPU tests (TESTS=0 skips), then bench lines for the given
# configs (default c2), no CPU baseline / drop-in e2e.  Logs in gpurun_out/q3_<tag>/.
#   tools/quick3.sh <tag> [configs...]
set -u
TAG=$1; shift
CFGS=${@:-c2}
OUT=gpurun_out/q3_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import json,sys; sys.path.insert(0,'.'); from tiny_mp2v_dec_amd import build as B; print('provenance:', json.dumps(B.provenance()))"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || { tail -30 $OUT/gpu_tests.log; exit 1; }
fi
for c in $CFGS; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --config $c ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python - $OUT/bench_$c.json $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = {k.split('<')[1].split('>')[0]: (v['avg_launch_ms'], v['frac']) for k, v in d['roofline']['per_kernel'].items()}
print(sys.argv[2], d['value'], 'frac', d['roofline']['frac'], d['parity']['status'], 'ms/step', d['ms_per_step'], pk)
PY
done

#!/bin/bash
# Round-4 evidence for the current build, one GPU call: GPU tests, smoke, the default bench line
# (c2 with the CPU baseline and the drop-in e2e), bench lines for the other configs, then the
# rocprofv3 kernel trace + FETCH/WRITE/TCC passes of the c2 and c5 bench commands (the
# roofline.traffic of their lines: tools/prof_summary.py --json).  Logs in gpurun_out/r4_<tag>/.
#   tools/r4_evidence.sh <tag>          (CONFIGS="c1 c3 c4 c5", PROFILE="c2 c5" to narrow)
set -u
TAG=$1
OUT=gpurun_out/r4_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROV=$(python -c "import json,sys; sys.path.insert(0,'.'); from tiny_mp2v_dec_amd import build as B; print(json.dumps(B.provenance()))")
echo "provenance: $PROV"
stamp() { echo "# provenance: $PROV" > "$1"; }
if [ "${TESTS:-1}" = 1 ]; then
  stamp $OUT/gpu_tests.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread >> $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || exit 1
  stamp $OUT/smoke.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  echo "$(tail -1 $OUT/smoke.log)"
fi
timeout -k 10 600 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
echo "c2: $(tail -1 $OUT/bench_c2.json | head -c 300)"
for c in ${CONFIGS:-c1 c3 c4 c5}; do
  extra="--no-cpu-baseline --no-e2e"
  [ $c = c1 ] && extra="--no-e2e"
  timeout -k 10 400 python bench.py $extra --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  echo "$c: $(tail -1 $OUT/bench_$c.json | head -c 200)"
done
if [ "${E2E1:-1}" = 1 ]; then  # the drop-in and the reference at one host thread (verdict r3 item 6)
  timeout -k 10 600 python tools/e2e_bench.py --threads 1 --ref --gops 8 > $OUT/e2e_1thread.json 2> $OUT/e2e_1thread.err || { tail -5 $OUT/e2e_1thread.err; exit 1; }
  echo "e2e 1 thread: $(tail -1 $OUT/e2e_1thread.json)"
fi
for c in ${PROFILE:-c2 c5}; do
  PASSES=traffic tools/profile.sh ${TAG}_$c --config $c --steps 10 --warmup 2 --no-e2e > $OUT/profile_$c.log 2>&1 || { cat $OUT/profile_$c.log; exit 1; }
  echo "profile $c ok"
done

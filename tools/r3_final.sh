#!/bin/bash
# Round-3 evidence for the current build: GPU tests, smoke, the default bench line (CPU baseline +
# drop-in e2e), bench lines for c1/c3/c4/c5, and (optional, PROFILE=1) the single-stream rocprofv3
# kernel trace + PMC passes of the c2 bench command.  Logs in gpurun_out/r3f_<tag>/; every log
# starts with the provenance line (git commit recorded by build(), libmp2vg content stamp).
set -u
TAG=$1
OUT=gpurun_out/r3f_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROV=$(python -c "import json,sys; sys.path.insert(0,'.'); from tiny_mp2v_dec_amd import build as B; print(json.dumps(B.provenance()))")
echo "provenance: $PROV"
stamp() { echo "# provenance: $PROV" > "$1"; }
stamp $OUT/gpu_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread >> $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || exit 1
stamp $OUT/smoke.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
echo "$(tail -1 $OUT/smoke.log)"
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
echo "c2: $(tail -1 $OUT/bench_c2.json | head -c 300)"
for c in ${CONFIGS:-c1 c3 c4 c5}; do
  extra="--no-cpu-baseline --no-e2e"
  [ $c = c1 ] && extra="--no-e2e"
  timeout -k 10 400 python bench.py $extra --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  echo "$c: $(tail -1 $OUT/bench_$c.json | head -c 200)"
done
if [ "${PROFILE:-0}" = 1 ]; then
  MP2VG_STREAMS=1 tools/profile.sh ${TAG}_s1 --steps 10 --warmup 2 --no-e2e > $OUT/profile_s1.log 2>&1 || { cat $OUT/profile_s1.log; exit 1; }
  echo "profile (1 stream) ok"
fi

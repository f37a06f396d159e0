#!/bin/bash
# Round-2 evidence for the current build: GPU tests, the default bench line (CPU baseline +
# drop-in e2e), bench lines for c3/c4/c5, and the single-stream rocprofv3 kernel trace + PMC
# passes of the c2 bench command.  Logs in gpurun_out/r2f_<tag>/.
set -u
TAG=$1
OUT=gpurun_out/r2f_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
echo "$(tail -1 $OUT/smoke.log)"
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
echo "c2: $(tail -1 $OUT/bench_c2.json | head -c 300)"
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  echo "$c: $(tail -1 $OUT/bench_$c.json | head -c 200)"
done
MP2VG_STREAMS=1 tools/profile.sh ${TAG}_s1 --steps 10 --warmup 2 --no-e2e > $OUT/profile_s1.log 2>&1 || { cat $OUT/profile_s1.log; exit 1; }
echo "profile (1 stream) ok"
tools/profile.sh ${TAG}_s2 --steps 10 --warmup 2 --no-e2e > $OUT/profile_s2.log 2>&1 || { cat $OUT/profile_s2.log; exit 1; }
echo "profile (2 streams) ok"

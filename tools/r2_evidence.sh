#!/bin/bash
# Round-2 evidence on the GPU box: GPU tests, the default bench line, and a single-stream
# (MP2VG_STREAMS=1) rocprofv3 kernel trace + FETCH/WRITE passes of the same bench command, so the
# per-kernel average launch time is not inflated by two-stream overlap.  Logs in gpurun_out/r2_<tag>/.
#   tools/r2_evidence.sh <tag> [notests]
set -u
TAG=$1; MODE=${2:-all}
OUT=gpurun_out/r2_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" != notests ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/gpu_tests.log)"; [ $rc = 0 ] || exit 1
fi
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
echo "c2: $(tail -1 $OUT/bench_c2.json | head -c 400)"
MP2VG_STREAMS=1 tools/profile.sh ${TAG}_s1 --steps 10 --warmup 2 --no-e2e > $OUT/profile_s1.log 2>&1 || { cat $OUT/profile_s1.log; exit 1; }
echo "profile (1 stream) ok"
MP2VG_STREAMS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2 > $OUT/bench_c2_s1.json 2> $OUT/bench_c2_s1.err || exit 1
echo "c2 1-stream: $(tail -1 $OUT/bench_c2_s1.json | head -c 300)"

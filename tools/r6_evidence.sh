#!/bin/bash
# Round-6 evidence for the current build (run on the GPU box via gpurun), in two parts so each
# call stays well inside gpurun's limit.  Logs in gpurun_out/r6_<tag>/.
#   PART=bench tools/r6_evidence.sh <tag>   GPU tests, smoke, bench lines c2 (CPU baseline + drop-in
#                                           e2e) and c1 c3 c4 c5 (TESTS=0 skips the tests)
#   PART=prof  tools/r6_evidence.sh <tag>   one-stream rocprofv3 summaries (tools/pmc5.sh) of c2 and
#                                           c5, and the bench commands' FETCH/WRITE traffic passes
#                                           (tools/profile.sh, bench.py roofline.traffic)
set -u
TAG=$1
OUT=gpurun_out/r6_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROV=$(python -c "import json,sys; sys.path.insert(0,'.'); from tiny_mp2v_dec_amd import build as B; print(json.dumps(B.provenance()))")
echo "provenance: $PROV"
stamp() { echo "# provenance: $PROV" > "$1"; }
if [ "${PART:-bench}" = bench ]; then
  if [ "${TESTS:-1}" = 1 ]; then
    stamp $OUT/gpu_tests.log
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread >> $OUT/gpu_tests.log 2>&1
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
else
  CFG=c2 tools/pmc5.sh ${TAG}_c2 > $OUT/pmc5_c2.txt 2>&1 || { tail -5 $OUT/pmc5_c2.txt; exit 1; }
  echo "pmc5 c2 ok"
  CFG=c5 PMC_GROUPS="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
    tools/pmc5.sh ${TAG}_c5 > $OUT/pmc5_c5.txt 2>&1 || { tail -5 $OUT/pmc5_c5.txt; exit 1; }
  echo "pmc5 c5 ok"
  for c in ${PROFILE:-c2 c5}; do
    PASSES=traffic tools/profile.sh ${TAG}_$c --config $c --steps 10 --warmup 2 --no-e2e > $OUT/profile_$c.log 2>&1 || { cat $OUT/profile_$c.log; exit 1; }
    echo "profile $c ok"
  done
fi

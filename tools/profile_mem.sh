#!/bin/bash
# Memory-pipeline counters (TA / TCP / UTCL1 / TD) of the recon kernel, one rocprofv3 pass per
# counter group (run on the GPU box):  tools/profile_mem.sh <tag> [bench args...]
set -u
TAG=$1; shift
ARGS="$@"
OUT=gpurun_out/profm_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run ta1 TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum || exit 1
run ta2 TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum || exit 1
run tcp1 TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum || exit 1
run tcp2 TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum || exit 1
run tcp3 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || exit 1
run utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum || exit 1
run utcl2 TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum || exit 1
run utcl3 TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum || exit 1
run lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum || exit 1
run gui GRBM_GUI_ACTIVE TA_BUSY_avr || exit 1
echo done

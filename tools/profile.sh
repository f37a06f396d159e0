#!/bin/bash
# Collect the rocprofv3 evidence for one bench configuration (run on the GPU box via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Pass 1: kernel trace + stats (same command as the bench);  passes 2+: PMC counters, each in
# its own run with --kernel-trace only (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not
# fit one pass).  Raw output lands in gpurun_out/prof_<tag>/.
set -u
TAG=$1; shift
ARGS="$@"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run ktrace --kernel-trace --stats || exit 1
run fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run write --kernel-trace --pmc WRITE_SIZE || exit 1
[ "${PASSES:-all}" = traffic ] && { run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1; echo done; exit 0; }
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES || exit 1
run sq2 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM || exit 1
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
echo done

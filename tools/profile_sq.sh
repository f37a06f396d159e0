#!/bin/bash
# Shader-issue counters (VALU / LDS / wait) of the recon kernels, one rocprofv3 pass per counter
# pair (run on the GPU box):  tools/profile_sq.sh <tag> [bench args...]
set -u
TAG=$1; shift
ARGS="$@"
OUT=gpurun_out/profq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run q1 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES || exit 1
run q2 SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
run q3 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit 1
run q4 SQ_INSTS_LDS SQ_ACTIVE_INST_LDS || exit 1
run q5 SQ_INSTS_SALU SQ_WAVES || exit 1
echo done

#!/bin/bash
# GPU parity tests of the in-tree build, then an interleaved bench A/B against variant libraries
#   tools/test_and_ab.sh <tag> "<bench args>" <rounds> <variant>...
TAG=$1; ARGS=$2; R=$3; shift 3
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/$TAG/gpu_tests.log)"
if [ $rc != 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/$TAG/gpu_tests.log | head -20; exit 1; fi
tools/ab_lib.sh "$ARGS" $R "$@"

#!/bin/bash
# GPU tests, then interleaved A/B of the in-tree build against one variant on c2 and c5
#   tools/ab2.sh <tag> <variant> <rounds>
TAG=$1; V=$2; R=$3
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/$TAG/gpu_tests.log)"
if [ $rc != 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/$TAG/gpu_tests.log | head -20; exit 1; fi
for cfg in ${CFGS:-c2 c5}; do
  tools/ab_lib.sh "--config $cfg --steps 10 --no-e2e" $R $V | sed "s/^/$cfg /" || exit 1
done

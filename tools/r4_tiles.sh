#!/bin/bash
# anchor tiles: GPU tests of the in-tree build, then same-box A/B against the pre-tile library
# (_var/base0) on every config.  Logs in gpurun_out/r4t/.
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4t/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r4t/gpu_tests.log)"; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4t/gpu_tests.log | head -20; exit 1; }
tools/ab_cfg_env.sh "${CFGS:-c2 c3 c1 c5 c4}" ${R:-2} "--steps 8" base base0 > gpurun_out/r4t/ab.log 2>&1; rc=$?
cat gpurun_out/r4t/ab.log; exit $rc

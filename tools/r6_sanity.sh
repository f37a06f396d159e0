#!/bin/bash
# Round-6 last sanity (gpurun): GPU tests and smoke on the committed build
set -o pipefail
mkdir -p gpurun_out/r6_sanity
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_sanity/gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6_sanity/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_sanity/smoke.log 2>&1 || { tail -5 gpurun_out/r6_sanity/smoke.log; exit 1; }
tail -1 gpurun_out/r6_sanity/smoke.log
echo ALL_DONE

#!/bin/bash
# Effective shader clock of the recon kernels: GRBM_GUI_ACTIVE cycles / kernel-trace duration.
set -u
OUT=gpurun_out/profc_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/c -o c -- python3 bench.py --no-cpu-baseline "$@" > $OUT/c.log 2>&1
echo "rc=$?"

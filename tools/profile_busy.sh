#!/bin/bash
# Derived busy metrics of the recon kernels (one rocprofv3 pass each) + the available counter list.
set -u
OUT=gpurun_out/profb_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
for m in VALUBusy VALUUtilization SALUBusy LDSBankConflict MemUnitBusy; do
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc $m --output-format csv -d $OUT/$m -o $m -- python3 bench.py --no-cpu-baseline "$@" > $OUT/$m.log 2>&1
  echo "$m rc=$?"
done

#!/bin/bash
# Dynamic instruction counts of the recon kernels under each ablation (dev tool, GPU box).
export MP2VG_LIB=${MP2VG_LIB:-tiny_mp2v_dec_amd/_var/dev/libmp2vg.so}  # tools/dev_build.sh
set -u
OUT=gpurun_out/profa_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for a in 0 1 2 4 32 64; do
  MP2VG_ABLATE=$a timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/a$a -o a$a -- python3 tools/launch_breakdown.py --gops 32 > $OUT/a$a.log 2>&1 || exit 1
  echo "abl $a ok"
done

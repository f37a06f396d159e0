#!/bin/bash
# Stage stamps of dev builds, then an interleaved bench A/B (run on the GPU box via gpurun).
#   STAMPS="dev devhead" AB="base v5 head" ROUNDS=2 CFG=c2 tools/stamps_ab.sh <tag>
set -o pipefail
TAG=$1
CFG=${CFG:-c2}
for v in ${STAMPS:-}; do
  MP2VG_LIB=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so MP2VG_ABLATE=16 timeout -k 10 240 python tools/stamps.py --config $CFG --gops 32 \
    > gpurun_out/stamps_${TAG}_$v.txt 2>&1 || { echo "stamps $v failed"; exit 1; }
done
[ -n "${AB:-}" ] && { CFG=$CFG timeout -k 10 1000 tools/ab5.sh ${ROUNDS:-2} $AB > gpurun_out/ab_${TAG}.txt 2>&1 || exit 1; }
echo done

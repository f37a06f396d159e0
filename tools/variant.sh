#!/bin/bash
# Build an A/B variant of the library from a patched recon.hip into tiny_mp2v_dec_amd/_var/<name>/
#   tools/variant.sh <name> <patched recon.hip>
set -e
NAME=$1; SRC=$2
OUT=tiny_mp2v_dec_amd/_var/$NAME
mkdir -p $OUT
cp tiny_mp2v_dec_amd/_build/*.o $OUT/ 2>/dev/null || true
hipcc -x hip --offload-arch=gfx950 -munsafe-fp-atomics ${EXTRA:-} -O3 -fPIC -std=c++17 -I tiny_mp2v_dec_amd/csrc -I include -c $SRC -o $OUT/recon.hip.o
hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libmp2vg.so $OUT/*.o -lpthread
echo $OUT/libmp2vg.so

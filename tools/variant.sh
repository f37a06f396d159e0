#!/bin/bash
# Build an A/B variant of the library from a patched recon.hip into tiny_mp2v_dec_amd/_var/<name>/
# and print the VGPR / scratch / occupancy of its 4:2:0 kernels (a variant that spills is suspect)
#   tools/variant.sh <name> <patched recon.hip>
set -e
NAME=$1; SRC=$2
OUT=tiny_mp2v_dec_amd/_var/$NAME
mkdir -p $OUT
cp tiny_mp2v_dec_amd/_build/*.o $OUT/ 2>/dev/null || true
hipcc -x hip --offload-arch=gfx950 -munsafe-fp-atomics ${EXTRA:-} -O3 -fPIC -std=c++17 -I tiny_mp2v_dec_amd/csrc -I include -c $SRC -o $OUT/recon.hip.o -Rpass-analysis=kernel-resource-usage 2> $OUT/resource.txt
# dev builds (EXTRA=-DMP2VG_DEV_ABLATIONS): runtime.cpp's dev_env knobs too
if [[ "${EXTRA:-}" == *MP2VG_DEV_ABLATIONS* ]]; then
  hipcc -D__HIP_PLATFORM_AMD__ $EXTRA -w -O3 -fPIC -std=c++17 -I tiny_mp2v_dec_amd/csrc -I include -c tiny_mp2v_dec_amd/csrc/runtime.cpp -o $OUT/runtime.cpp.o
fi
hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libmp2vg.so $OUT/*.o -lpthread
python3 - $OUT/resource.txt $NAME <<'PY'
import re, sys
cur = None; res = {}
for l in open(sys.argv[1]):
    m = re.search(r"Function Name: _ZN5mp2vg12recon_kernelILi(\d)ELi(\d)ELi0E", l)
    if m: cur = f"<{m.group(1)},{m.group(2)}>"; res[cur] = {}; continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", l)
    if m and cur: res[cur][m.group(1).split()[0]] = int(m.group(2))
print(sys.argv[2], " ".join(f"{k}:{v.get('VGPRs')}v/{v.get('ScratchSize')}s/{v.get('Occupancy')}w" for k, v in sorted(res.items())))
PY

#!/bin/bash
# Round-6 placement probe 3 (gpurun, one box): the 6-context placement probe (tools/placement.py)
# once per pool allocation setting, e.g. tools/r6_placement3.sh MP2VG_POOL_CHUNK=64 MP2VG_POOL_CHUNK=0
set -o pipefail
mkdir -p gpurun_out
for arm in "$@"; do
  tag=$(echo "$arm" | tr '=@,/' '____')
  env ${arm//,/ } timeout -k 10 300 python -u tools/placement.py --config c2 --contexts 6 --steps 10 --reps 1 > gpurun_out/placement3_$tag.txt 2>&1 || { tail -5 gpurun_out/placement3_$tag.txt; exit 1; }
  echo "== $arm"; grep -v '^{' gpurun_out/placement3_$tag.txt | grep -v "rw frames\|ro frames\|per-block"
done
echo ALL_DONE

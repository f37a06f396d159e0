#!/bin/bash
# Round-6: drop-in host frames, the download path: copy kernel with 64 (default) / 256 workgroups
# per chunk, or one DMA per frame (MP2VG_DL_KERNEL=0); one process per arm, 3 back-to-back calls,
# interleaved twice
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for arm in "MP2VG_DL_WGS=64" "MP2VG_DL_WGS=256" "MP2VG_DL_KERNEL=0"; do
    env $arm timeout -k 10 300 python -u tools/dropin_trace.py 256 host 3 16 > gpurun_out/dl.jsonl 2>/dev/null || exit 1
    echo "$arm round $r: $(python3 -c "import json,sys; print([(d['frames_per_s'], d['cpus_busy']) for d in map(json.loads, open(sys.argv[1]))])" gpurun_out/dl.jsonl)"
  done
done
echo ALL_DONE

#!/bin/bash
# Round-6: drop-in host frames, blocking download waits (default) vs spinning (MP2VG_DL_BLOCKING=0),
# one process per arm, 3 back-to-back decode() calls each, arms interleaved twice
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for b in 1 0; do
    MP2VG_DL_BLOCKING=$b timeout -k 10 300 python -u tools/dropin_trace.py 256 host 3 16 > gpurun_out/dropin_blk${b}_$r.jsonl 2>/dev/null || exit 1
    echo "blocking=$b round $r: $(python3 -c "import json,sys; print([(d['frames_per_s'], d['cpus_busy']) for d in map(json.loads, open(sys.argv[1]))])" gpurun_out/dropin_blk${b}_$r.jsonl)"
  done
done
echo ALL_DONE

#!/bin/bash
# Round-6: drop-in decode() threads on the GPU's NUMA node (MP2VG_PIN=1, default) or anywhere
# (MP2VG_PIN=0): back-to-back calls, both frame modes, one process per arm, interleaved twice
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for pin in 1 0; do
    MP2VG_PIN=$pin timeout -k 10 300 python -u tools/dropin_trace.py 256 both 3 16 > gpurun_out/dropin_pin${pin}_$r.jsonl 2>/dev/null || exit 1
    echo "pin=$pin round $r: $(python3 -c "import json,sys; print([(('dev' if d['device_frames'] else 'host'), d['frames_per_s'], d['cpus_busy']) for d in map(json.loads, open(sys.argv[1]))])" gpurun_out/dropin_pin${pin}_$r.jsonl)"
  done
done
echo ALL_DONE

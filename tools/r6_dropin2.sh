#!/bin/bash
# Round-6: drop-in end to end, back-to-back decode() calls on one decoder per frame mode (as the
# bench's e2e lines run them), with the native phase trace (gpurun)
set -o pipefail
mkdir -p gpurun_out
for m in host device; do
  MP2VG_TRACE=1 timeout -k 10 300 python -u tools/dropin_trace.py 256 $m 3 > gpurun_out/dropin_b2b_$m.jsonl 2> gpurun_out/dropin_b2b_${m}_trace.txt || { tail -20 gpurun_out/dropin_b2b_${m}_trace.txt; exit 1; }
  cat gpurun_out/dropin_b2b_$m.jsonl
  grep -E "^=== |\(sum\)|after parse|headers" gpurun_out/dropin_b2b_${m}_trace.txt | head -40
done
echo ALL_DONE

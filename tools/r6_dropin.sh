#!/bin/bash
# Round-6: drop-in end to end, host frames vs device frames, interleaved runs on one box with the
# native phase trace (gpurun)
set -o pipefail
mkdir -p gpurun_out
MP2VG_TRACE=1 timeout -k 10 600 python -u tools/dropin_trace.py 256 both 3 > gpurun_out/dropin_modes.jsonl 2> gpurun_out/dropin_modes_trace.txt || { tail -20 gpurun_out/dropin_modes_trace.txt; exit 1; }
cat gpurun_out/dropin_modes.jsonl
grep -E "^=== |\(sum\)|after parse" gpurun_out/dropin_modes_trace.txt | head -80

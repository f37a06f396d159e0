#!/bin/bash
# Round-6: drop-in back-to-back decode() calls, host frames then device frames (4 runs each, 16
# threads), with the process's CPU use per run (cpus_busy = CPU seconds / wall seconds)
set -o pipefail
mkdir -p gpurun_out
for m in host device; do
  MP2VG_TRACE=1 timeout -k 10 300 python -u tools/dropin_trace.py 256 $m 4 16 > gpurun_out/dropin_cpu_$m.jsonl 2> gpurun_out/dropin_cpu_${m}_trace.txt || { tail -20 gpurun_out/dropin_cpu_${m}_trace.txt; exit 1; }
  cat gpurun_out/dropin_cpu_$m.jsonl
  grep -E "parse wait|download wait" gpurun_out/dropin_cpu_${m}_trace.txt | tr -s ' ' | tr '\n' ';'; echo
done
echo ALL_DONE

#!/bin/bash
# Round-6: drop-in back-to-back decode() calls (device frames, 4 runs) at several host thread
# counts, under the box's CPU quota (cpu.max), with the native phase trace (gpurun)
set -o pipefail
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max
for t in "$@"; do
  MP2VG_TRACE=1 timeout -k 10 300 python -u tools/dropin_trace.py 256 device 4 $t > gpurun_out/dropin_thr_$t.jsonl 2> gpurun_out/dropin_thr_${t}_trace.txt || { tail -20 gpurun_out/dropin_thr_${t}_trace.txt; exit 1; }
  cat gpurun_out/dropin_thr_$t.jsonl
  grep -E "parse wait" gpurun_out/dropin_thr_${t}_trace.txt | tr '\n' ' '; echo
done
echo ALL_DONE

#!/bin/bash
# Round-6: an uncalibrated one-stream context with device memory allocated after its pool and held
# (0 / 29 / 58 GB), 2 interleaved rounds: does memory allocated after a pool change its speed?
set -o pipefail
for r in 1 2; do
  for gb in 0 29 58; do
    MP2VG_PLACE_CANDIDATES=1 timeout -k 10 200 python -u tools/onestream.py --config c2 --reps 5 --ballast-after-gb $gb > gpurun_out/ba.json 2>&1 || { tail -3 gpurun_out/ba.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ballast-after', sys.argv[2], 'GB | span', d['span_ms'])" gpurun_out/ba.json $gb
  done
done
echo ALL_DONE

#!/bin/bash
# Round-6: does a calibrated one-stream context run slow right after its calibration (freed
# candidate pools cleared in the background?) -- onestream.py with the calibration on, timed
# batches right after it or after a 2-s pause, interleaved
set -o pipefail
for r in 1 2; do
  for sl in 0 2; do
    MP2VG_PLACE_ONE_STREAM=1 timeout -k 10 200 python -u tools/onestream.py --config c2 --reps 5 --sleep $sl > gpurun_out/place_sleep_${sl}_$r.json 2>&1 || { tail -3 gpurun_out/place_sleep_${sl}_$r.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('sleep', sys.argv[2], 'span', d['span_ms'], 'calib', d['pool_placement'])" gpurun_out/place_sleep_${sl}_$r.json $sl
  done
  timeout -k 10 200 python -u tools/onestream.py --config c2 --reps 5 > gpurun_out/place_sleep_off_$r.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('uncalibrated span', d['span_ms'])" gpurun_out/place_sleep_off_$r.json
done
echo ALL_DONE

#!/bin/bash
# Round-6: the calibrated one-stream context's slow batches: discarded candidate pools held until
# destroy (MP2VG_PLACE_HOLD=1), or freed and a 10-s pause, against no calibration; interleaved
set -o pipefail
for r in 1 2; do
  for arm in "MP2VG_PLACE_ONE_STREAM=1 MP2VG_PLACE_HOLD=1 --sleep 0" "MP2VG_PLACE_ONE_STREAM=1 --sleep 10" "MP2VG_PLACE_CANDIDATES=1 --sleep 0"; do
    envs=${arm%%--*}; args=--${arm#*--}
    env $envs timeout -k 10 200 python -u tools/onestream.py --config c2 --reps 5 $args > gpurun_out/place_hold.json 2>&1 || { tail -3 gpurun_out/place_hold.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '| span', d['span_ms'], 'calib', d['pool_placement'])" gpurun_out/place_hold.json "$arm"
  done
done
echo ALL_DONE

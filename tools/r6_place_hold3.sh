#!/bin/bash
# Round-6: c2 bench, placement calibration (held candidates, one-stream contexts too: the new
# default) against none; 3 interleaved rounds; then the one-stream tool's calibrated context
set -o pipefail
ROUNDS=1 bash tools/ab5.sh 3 base base@MP2VG_PLACE_CANDIDATES=1 > gpurun_out/ab_r6_place_hold3.txt || { cat gpurun_out/ab_r6_place_hold3.txt; exit 1; }
cat gpurun_out/ab_r6_place_hold3.txt
for r in 1 2; do
  timeout -k 10 200 python -u tools/onestream.py --config c2 --reps 5 > gpurun_out/os_hold.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('onestream span', d['span_ms'], d['pool_placement'], {k: v['avg_launch_ms'] for k, v in d['per_kernel'].items()})" gpurun_out/os_hold.json
done
echo ALL_DONE

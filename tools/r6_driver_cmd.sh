#!/bin/bash
# Round-6: the driver's own bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) once
# on this box; the JSON line to gpurun_out/driver_cmd_<tag>.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_cmd_$1.json 2> gpurun_out/driver_cmd_$1.err || { tail -5 gpurun_out/driver_cmd_$1.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['frac'], d['parity']['status'], 'span1', r['one_stream_span_ms'], d['pool_placement']['candidate_batch_ms'], d['pool_placement']['kept'], 'e2e', d['e2e_dropin']['runs_frames_per_s'], d['e2e_dropin_device_frames']['runs_frames_per_s'], 'cpu', d['cpu_baseline']['value'], d['box'])" gpurun_out/driver_cmd_$1.json
echo ALL_DONE

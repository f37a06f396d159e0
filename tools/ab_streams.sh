# GPU tests, then bench with 1..4 independent picture-set streams (MP2VG_STREAMS)
set -e
mkdir -p gpurun_out/streams
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/streams/tests.log 2>&1 || { tail -30 gpurun_out/streams/tests.log; exit 1; }
tail -1 gpurun_out/streams/tests.log
for n in ${NS:-1 2 3 4 1 2}; do
  MP2VG_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/streams/s$n.json 2> gpurun_out/streams/s$n.err
  echo "streams=$n $(python3 -c "import json;d=json.loads(open('gpurun_out/streams/s$n.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['frame_digest_of_digests'])")"
done

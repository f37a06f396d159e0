"""Drop-in end to end, repeated, with the native phase trace (dev tool, run on the GPU box): the c2
bench stream (64 GOPs) decoded 6 times by one mp2v_decoder_c per frame mode (host frames, and
with `both` also device frames, MP2VG_DECODER_DEVICE_FRAMES; 16 threads), runs of the two modes
interleaved; prints frames/s per run, and MP2VG_TRACE's per-phase lines go to stderr, for telling
a slow run's phase.

    MP2VG_TRACE=1 python tools/dropin_trace.py [gops] [host|device|both] [runs] [threads] 2> trace.txt
"""
import json
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402
from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 64
modes = {"host": [False], "device": [True], "both": [False, True]}[sys.argv[2] if len(sys.argv) > 2 else "host"]
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 6
threads = int(sys.argv[4]) if len(sys.argv) > 4 else 16
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
n = [0]
decs = {m: mp2v_decoder_c(decoder_config_t(w, h, cf, pictures_pool_size=24, num_threads=threads, device_frames=m),
                          lambda f: n.__setitem__(0, n[0] + 1)) for m in modes}
for run in range(runs):
    for m in modes:
        n[0] = 0
        print(f"=== run {run} {'device' if m else 'host'} frames", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        decs[m].decode(es)
        dt = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        print(json.dumps({"run": run, "threads": threads, "device_frames": m, "frames": n[0],
                          "frames_per_s": round(n[0] / dt, 1), "cpus_busy": round(cpu / dt, 2)}), flush=True)
for d in decs.values():
    d.close()

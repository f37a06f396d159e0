"""Multi-lane drop-in hand-off probe (dev tool, run on the GPU box): the c2 bench stream decoded by
mp2v_decoder_c over N lanes on the one GPU (devices [0] * N), host frames, a null renderer.

    python tools/handoff_probe.py [gops] [lanes...]

Prints per lane count: frames/s end to end, frames per lane, and decoder.cpp's hand-off stats
(lane changes that left the lane just left downloading -- its chunk in flight while the next
lane is fed -- and host waits on another lane forced by the frame pool).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402
from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 32
lanes = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 2)
for n in lanes:
    frames = [0]
    dec = mp2v_decoder_c(decoder_config_t(w, h, cf, num_threads=threads, devices=[0] * n),
                         lambda f: frames.__setitem__(0, frames[0] + 1))
    dec.decode(es)  # warm-up: pools, banks, streams
    frames[0] = 0
    t0 = time.perf_counter()
    dec.decode(es)
    dt = time.perf_counter() - t0
    stats = dec.handoff_stats()
    out = {"lanes": n, "frames": frames[0], "frames_per_s": round(frames[0] / dt, 1), "lane_frames": dec.lane_frames(),
           "handoffs_left_in_flight": stats[0], "host_waits_on_other_lane": stats[1],
           "handoffs_landed": stats[2], "lane_changes": stats[3],
           "frames_allocated": dec.frames_allocated(), "host_threads": threads}
    dec.close()
    print(json.dumps(out), flush=True)

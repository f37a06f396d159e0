"""Host record emitter throughput vs worker threads on the c2 bench stream (run on the GPU box's
host: the drop-in's parse runs there).

    python tools/parse_scale.py [gops] [threads...]

Times mp2vg_parse_es alone (start codes, headers, every slice's VLC -> records on `threads`
workers, coefficient concatenation), best of 3, and prints one JSON line per thread count plus
the parallel efficiency against one thread.  `slices_ms` is the worker phase alone (MP2VG_TRACE's
"parse: slices": the part that scales with workers, and the only part the drop-in decoder's
streaming parse runs -- it recycles its buffers and gathers records on helper threads, so it has
neither mp2vg_parse_es's serial buffer zeroing nor its concatenation).
"""
import ctypes
import json
import os
import sys
import tempfile
import time

os.environ["MP2VG_TRACE"] = "1"  # per-phase times on stderr (tables.cpp trace_phase), read below

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiny_mp2v_dec_amd import _lib  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 16
threads = [int(t) for t in sys.argv[2:]] or [1, 2, 4, 8, 14, 16]
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
buf = np.frombuffer(es, dtype=np.uint8)
frames = 12 * gops
base = None
for t in threads:
    cfg = _lib.make_config(w, h, cf, threads=t)
    best, best_sl = 1e9, 1e9
    for _ in range(3):
        hh = ctypes.c_void_p()
        with tempfile.TemporaryFile() as tf:
            saved = os.dup(2)
            os.dup2(tf.fileno(), 2)
            try:
                t0 = time.perf_counter()
                _lib.check(_lib.lib().mp2vg_parse_es(buf.ctypes.data_as(ctypes.c_void_p), len(es), ctypes.byref(cfg),
                                                     ctypes.byref(hh)), "parse_es")
                dt = time.perf_counter() - t0
            finally:
                os.dup2(saved, 2)
                os.close(saved)
            tf.seek(0)
            sl = [float(l.split()[-2]) for l in tf.read().decode().splitlines() if "parse: slices" in l]
        best = min(best, dt)
        best_sl = min(best_sl, sl[-1] / 1e3 if sl else 1e9)
        _lib.lib().mp2vg_parsed_free(hh)
    fps, sfps = frames / best, frames / best_sl
    base = base or (fps / t, sfps / t)
    print(json.dumps({"threads": t, "frames": frames, "ms": round(best * 1e3, 2), "frames_per_s": round(fps, 1),
                      "efficiency": round(fps / (base[0] * t), 3), "slices_ms": round(best_sl * 1e3, 2),
                      "slices_frames_per_s": round(sfps, 1), "slices_efficiency": round(sfps / (base[1] * t), 3)}),
          flush=True)

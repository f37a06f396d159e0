"""Single-thread (and N-thread) host parse rate, C level (dev tool):
    [MP2VG_LIB=<variant .so>] python tools/parse_bench.py [--gops 16] [--threads 1 14] [--reps 3]
Times mp2vg_parse_es alone (no Python copies) on the c2 stream; prints best-of-reps frames/s."""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from tiny_mp2v_dec_amd import _lib, records as R  # noqa: E402
from tiny_mp2v_dec_amd._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gops", type=int, default=16)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 14])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    w, h, cf, extra, _ = bench.CONFIGS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=a.gops, seed=1729, **extra)
    buf = np.frombuffer(es, dtype=np.uint8)
    frames = None
    out = {}
    for t in a.threads:
        best = 0.0
        for _ in range(a.reps):
            cfg = _lib.make_config(w, h, cf, threads=t)
            hnd = ctypes.c_void_p()
            t0 = time.perf_counter()
            rc = lib().mp2vg_parse_es(buf.ctypes.data_as(ctypes.c_void_p), len(es), ctypes.byref(cfg),
                                      ctypes.byref(hnd))
            dt = time.perf_counter() - t0
            if rc != 0:
                raise RuntimeError(f"parse_es rc {rc}")
            n = ctypes.c_int32()
            lib().mp2vg_parsed_counts(hnd, ctypes.byref(n), None, None)
            frames = n.value
            lib().mp2vg_parsed_free(hnd)
            best = max(best, frames / dt)
        out[t] = round(best, 1)
    print(" ".join(f"{t}t {v}" for t, v in out.items()), f"frames/s ({frames} frames)")


if __name__ == "__main__":
    main()

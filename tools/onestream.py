"""The bench batch on a one-stream context only (dev tool, run on the GPU box; profile target).

    python tools/onestream.py [--config c2] [--gops N] [--reps 5]

bench.py's timed region runs two picture sets on two streams and, after it, the same batch on a
one-stream context for its per-kernel roofline.  Profiling bench.py therefore mixes two launch
shapes per kernel (half-batch two-stream launches and full-batch one-stream launches).  This tool
runs ONLY the one-stream context (one launch per dependency level over the whole batch: c2 I 256
frames, B 512, P+B 3 x 768), so a rocprofv3 kernel trace of it has one launch shape per kernel and
its per-kernel means compare directly with the bench line's `per_kernel` (HIP events of the same
launches).  Prints the same per-kernel table from its own HIP events, as JSON.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--gops", type=int, default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sleep", type=float, default=0.0, help="host seconds between the warm-up batch and the timed ones")
    ap.add_argument("--ballast-after-gb", type=float, default=0.0,
                    help="device memory allocated (and touched) after the context's pool, held to the end")
    a = ap.parse_args()
    w, h, cf, extra, _ = bench.CONFIGS[a.config]
    gops = a.gops or bench.DEFAULT_GOPS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
    p = R.Parsed(es, w, h, cf, threads=min(8, os.cpu_count() or 1))
    of_pic, modes = R.plan_batch(w, h, cf, p.npics, p.pics, p.mbs, p.coefs, one_stream=True)
    launch_bytes = np.bincount(of_pic, weights=bench.per_picture_bytes(p), minlength=len(modes))
    ctx = R.DeviceContext(w, h, cf, slots=p.npics, one_stream=True)
    ctx.upload(p.pics, p.mbs, p.coefs)
    if a.ballast_after_gb > 0:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ballast = ctypes.c_void_p()
        nb = ctypes.c_size_t(int(a.ballast_after_gb * (1 << 30)))
        assert hip.hipMalloc(ctypes.byref(ballast), nb) == 0 and hip.hipMemset(ballast, 0, nb) == 0
    ctx.decode()  # warm-up batch (not in the table; with MP2VG_PLACE_ONE_STREAM=1 the placement calibration runs in it)
    ctx.synchronize()
    place_ms, place_kept = ctx.placement()
    if a.sleep > 0:
        import time
        time.sleep(a.sleep)
    for _ in range(a.reps):
        ctx.decode()
    ctx.synchronize()
    l1 = np.array([ctx.batch_times(back)[1] for back in range(a.reps)])
    span = float(np.mean([ctx.batch_times(back)[0] for back in range(a.reps)]))
    dig = ctx.digests(np.arange(p.npics))
    exp = bench.expected_digests(a.config, gops, 1729)
    ctx.close()
    out = {"config": a.config, "gops": gops, "frames": int(p.npics), "batches_decoded": a.reps + 1,
           "pool_placement": {"candidate_batch_ms": place_ms, "kept": place_kept},
           "span_ms": round(span, 4), "parity": None if exp is None else bool(np.array_equal(dig, exp)),
           "per_kernel": {}}
    for m in sorted(set(modes.tolist())):
        sel = modes == m
        ms = float(l1[:, sel].mean(axis=0).sum())
        n = int(sel.sum())
        nbytes = float(launch_bytes[sel].sum())
        out["per_kernel"][f"recon_kernel<{cf}, {m}, 0>"] = {
            "mode": ["I", "P / one-direction B", "B", "P+B", "I, tiles converted after"][m], "launches_per_batch": n, "avg_launch_ms": round(ms / n, 4),
            "algorithmic_bytes_per_launch": int(nbytes / n),
            "frac": round(nbytes / (ms / 1e3) / 1e9 / bench.HBM_PEAK_GBS, 4)}
    print(json.dumps(out), flush=True)
    if out["parity"] is False:
        sys.exit(3)


if __name__ == "__main__":
    main()

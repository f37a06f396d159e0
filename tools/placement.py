"""Pool-placement probe (GPU): several identical decode contexts held at once in one process, each
timed for a few back-to-back batches, round-robin, twice.  A context whose time differs from the
others' on every repetition differs by where its pool landed, not by when it ran.  Per context:
ms per batch (device span of the timed batches) and mean launch ms per kernel mode.

  python tools/placement.py [--config c2] [--contexts 4] [--steps 10] [--reps 2] [--one-stream]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--contexts", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--one-stream", action="store_true")
    ap.add_argument("--ballast-gb", type=float, default=0.0, help="device memory held before the first context")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--ballast-touch", action="store_true", help="memset the ballast before the contexts")
    ap.add_argument("--recreate", action="store_true", help="after rep 0 close context 0 and open one more")
    ap.add_argument("--dummy-streams", type=int, default=0, help="HIP streams created before the first context")
    ap.add_argument("--dummy-work", action="store_true", help="one memset on each dummy stream")
    ap.add_argument("--dummy-ctx", action="store_true", help="a small context created (and decoded once) first")
    a = ap.parse_args()
    if a.dummy_streams:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        held = [ctypes.c_void_p() for _ in range(a.dummy_streams)]
        buf = ctypes.c_void_p()
        hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(1 << 20))
        for st in held:
            hip.hipStreamCreateWithFlags(ctypes.byref(st), 1)
            if a.dummy_work:  # a stream takes its hardware queue at its first submission
                hip.hipMemsetAsync(buf, 0, ctypes.c_size_t(1 << 20), st)
        hip.hipDeviceSynchronize()
        print(f"{a.dummy_streams} dummy streams{' with work' if a.dummy_work else ''}", flush=True)
    if a.ballast_gb > 0:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ballast = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(ballast), ctypes.c_size_t(int(a.ballast_gb * (1 << 30))))
        if a.ballast_touch:
            rc |= hip.hipMemset(ballast, 0, ctypes.c_size_t(int(a.ballast_gb * (1 << 30))))
            rc |= hip.hipDeviceSynchronize()
        print(f"ballast {a.ballast_gb} GB at {ballast.value:#x} rc {rc}", flush=True)
    w, h, cf, gp, _ = bench.CONFIGS[a.config]
    gops = bench.DEFAULT_GOPS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **gp)
    parsed = R.Parsed(es, w, h, cf, threads=8)
    _, modes = R.plan_batch(w, h, cf, parsed.npics, parsed.pics, parsed.mbs, parsed.coefs,
                            one_stream=a.one_stream)
    ctxs = []
    if a.dummy_ctx:
        es0 = R.generate_es(width=176, height=144, chroma_format=1, n_gops=1, gop_n=6, gop_m=3, seed=4242)
        p0 = R.Parsed(es0, 176, 144, 1)
        dummy = R.DeviceContext(176, 144, 1, slots=p0.npics, device=0, one_stream=a.one_stream)
        dummy.upload(p0.pics, p0.mbs, p0.coefs)
        dummy.decode()
        dummy.synchronize()
        print("dummy context first", flush=True)
    for i in range(a.contexts):
        c = R.DeviceContext(w, h, cf, slots=parsed.npics, device=0, one_stream=a.one_stream)
        c.upload(parsed.pics, parsed.mbs, parsed.coefs)
        c.decode()
        c.synchronize()
        ctxs.append(c)
    ref = None
    rows = {i: [] for i in range(a.contexts)}
    for rep in range(a.reps):
        for i, c in (enumerate(ctxs) if rep % 2 == 0 else reversed(list(enumerate(ctxs)))):
            for _ in range(a.steps):
                c.decode()
            c.synchronize()
            span = c.batches_span(a.steps - 1, 0) / a.steps
            l = np.array([c.batch_times(b)[1] for b in range(a.steps)]).mean(axis=0)
            per_mode = {int(m): round(float(l[modes == m].sum()), 4) for m in sorted(set(modes.tolist()))}
            rows[i].append((round(span, 4), per_mode))
            print(f"rep {rep} ctx {i}: {span:.4f} ms/batch  per-mode launch ms {per_mode}", flush=True)
        if a.recreate and rep == 0:
            ctxs[0].close()
            c = R.DeviceContext(w, h, cf, slots=parsed.npics, device=0, one_stream=a.one_stream)
            c.upload(parsed.pics, parsed.mbs, parsed.coefs)
            c.decode()
            c.synchronize()
            ctxs[0] = c
            print("context 0 closed, a new context 0 opened", flush=True)
        d = ctxs[0].digests(np.arange(parsed.npics))
        for c in ctxs[1:]:
            if not np.array_equal(c.digests(np.arange(parsed.npics)), d):
                print("DIGEST MISMATCH between contexts")
                return 3
        ref = d
    # per-block HBM rate of each context's pool (frames and tiles blocks alternate)
    probe = {}
    for i, c in enumerate(ctxs):  # the record banks (cheap: one sweep each)
        rnd = [round(float(c.pool_probe(rw=2, reps=4)[0])) for _ in range(2)]
        lck = [round(float(c.pool_probe(rw=3, reps=4)[0])) for _ in range(2)]
        rndw = [round(float(c.pool_probe(rw=7, reps=4)[0])) for _ in range(2)]
        lckw = [round(float(c.pool_probe(rw=6, reps=4)[0])) for _ in range(2)]
        print(f"ctx {i} GB/s 1-KB runs: random {rnd} same-offset {lck} | stored back: random {rndw} "
              f"same-offset {lckw}", flush=True)
    for i, c in enumerate([] if a.no_probe else ctxs):
        rw = c.pool_probe(rw=1, reps=4)
        ro = c.pool_probe(rw=0, reps=4)
        probe[i] = {"rw_frames": rw[0::2].tolist(), "rw_tiles": rw[1::2].tolist(),
                    "ro_frames": ro[0::2].tolist(), "ro_tiles": ro[1::2].tolist()}
        def st(v):
            v = np.asarray(v)
            return f"mean {v.mean():7.1f} min {v.min():7.1f} p10 {np.percentile(v, 10):7.1f} max {v.max():7.1f}"
        print(f"ctx {i} probe GB/s  rw frames {st(rw[0::2])} | rw tiles {st(rw[1::2])}", flush=True)
        print(f"ctx {i} probe GB/s  ro frames {st(ro[0::2])} | ro tiles {st(ro[1::2])}", flush=True)
        rnd = [float(c.pool_probe(rw=2, reps=4)[0]) for _ in range(3)]
        lck = [float(c.pool_probe(rw=3, reps=4)[0]) for _ in range(3)]
        probe[i]["random_1k"], probe[i]["same_offset_1k"] = rnd, lck
        blk = c.pool_probe(rw=4, reps=2)
        probe[i]["block_random_frames"], probe[i]["block_random_tiles"] = blk[0::2].tolist(), blk[1::2].tolist()
        print(f"ctx {i} probe GB/s  per-block random: frames {st(blk[0::2])} | tiles {st(blk[1::2])}", flush=True)
        print(f"ctx {i} probe GB/s  random 1-KB reads {rnd}  same-offset 1-KB reads {lck}", flush=True)
    print(json.dumps({"config": a.config, "one_stream": a.one_stream, "contexts": a.contexts,
                      "ms_per_batch": {i: [r[0] for r in rows[i]] for i in rows}, "probe": probe}))
    for c in ctxs:
        c.close()
    return 0 if ref is not None else 1


if __name__ == "__main__":
    sys.exit(main())

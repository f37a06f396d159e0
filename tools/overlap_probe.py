"""Dev probe: how much do two independent batches gain from running concurrently (two device
contexts, two streams) instead of back to back?  Upper bound for cross-batch pipelining."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

w, h, cf, extra, _ = bench.CONFIGS["c2"]
ps = []
for seed in (1729, 1730):
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=32, seed=seed, **extra)
    ps.append(R.Parsed(es, w, h, cf, threads=8))
ctxs = [R.DeviceContext(w, h, cf, slots=p.npics) for p in ps]
for c, p in zip(ctxs, ps):
    c.upload(p.pics, p.mbs, p.coefs)
for c in ctxs:
    c.decode()
    c.synchronize()
for mode in ("sequential", "concurrent", "sequential", "concurrent"):
    t = time.perf_counter()
    for _ in range(10):
        if mode == "sequential":
            for c in ctxs:
                c.decode()
                c.synchronize()
        else:
            for c in ctxs:
                c.decode()
            for c in ctxs:
                c.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"{mode}: {dt * 1000:.3f} ms per pair of 384-frame batches")

"""Does a frame pool's placement change the kernels' speed?  Two contexts with the same batch held
at once, timed alternately (A, B, A, B), then both freed and two fresh ones made; per context the
ms per step and the summed launch ms per step (HIP events).  Same-box, same-process evidence for
run-to-run spreads that the launch schedule does not explain (dev tool).
    python tools/pool_var.py [config] [trials]"""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w, h, cf, gp, _ = bench.CONFIGS[cfg]
gops = bench.DEFAULT_GOPS[cfg]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **gp)
parsed = R.Parsed(es, w, h, cf, threads=8)
steps = 6


def timed(ctx):
    ctx.decode()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.decode()
    ctx.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    per = [ctx.batch_times(b)[1] for b in range(steps)]
    launch = sum(sum(x) for x in per) / steps
    each = [sum(x[i] for x in per) / steps for i in range(len(per[0]))]  # per launch (I, P+B, B+P, B+P, B)
    return ms, launch, each


for t in range(trials):
    ctxs = []
    for _ in range(2):
        c = R.DeviceContext(w, h, cf, slots=parsed.npics, device=0, one_stream=True)
        c.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctxs.append(c)
    for rep in range(2):
        for name, c in zip("AB", ctxs):
            ms, launch, each = timed(c)
            print(f"trial {t} ctx {name} rep {rep}: {ms:.3f} ms/step, launches {launch:.3f} ms/step "
                  f"({' '.join(f'{x:.3f}' for x in each)})", flush=True)
    for c in ctxs:
        c.close()

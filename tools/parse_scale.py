"""Host record emitter throughput vs worker threads (mp2vg_parse_es on the c2 bench stream).
    python tools/parse_scale.py [gops] [threads...]"""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 16
threads = [int(t) for t in sys.argv[2:]] or [1, 2, 4, 8, 16]
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
for t in threads:
    best = 0
    for _ in range(2):
        t0 = time.time()
        p = R.Parsed(es, w, h, cf, threads=t)
        best = max(best, p.npics / (time.time() - t0))
    print(t, round(best, 1), "frames/s", flush=True)

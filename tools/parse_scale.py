import time, sys
sys.path.insert(0, ".")
import bench
from tiny_mp2v_dec_amd import records as R
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=16, seed=1729, **extra)
for t in (1, 16, 1, 16):
    t0 = time.time(); p = R.Parsed(es, w, h, cf, threads=t); dt = time.time() - t0
    print(t, round(192 / dt, 1), "frames/s", flush=True)

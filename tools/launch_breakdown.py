"""Per-launch device times of one bench batch, by picture type (dev tool, run on the GPU box).

    python tools/launch_breakdown.py [--gops 32] [--reps 5] [--config c2]
Prints one line per launch: mcm (0 I / 1 P / 2 B), pictures, MBs, mean ms, us per 1k MBs.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gops", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    w, h, cf, extra, _ = bench.CONFIGS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=a.gops, seed=1729, **extra)
    p = R.Parsed(es, w, h, cf)
    with R.DeviceContext(w, h, cf, p.npics) as d:
        d.upload(p.pics, p.mbs, p.coefs)
        times = []
        for _ in range(a.reps + 1):
            d.decode()
            d.synchronize()
            times.append(d.launch_times_ms())
            spans = getattr(main, "spans", [])
            spans.append(d.batch_time_ms())
            main.spans = spans
        t = np.array(times[1:]).mean(axis=0)
        print(f"batch span {np.mean(main.spans[1:]):.4f} ms")
    # reconstruct the runtime's launch order: by dependency level, then I / P / B
    pct = p.pics["picture_coding_type"]
    mbs_per_pic = len(p.mbs) // p.npics
    print(f"launches {len(t)}  total {t.sum():.4f} ms  pictures {p.npics}")
    for i, ms in enumerate(t):
        print(f"launch {i}: {ms:.4f} ms")
    for c, name in ((1, "I"), (2, "P"), (3, "B")):
        print(f"{name}: {int(np.sum(pct == c))} pictures, {int(np.sum(pct == c)) * mbs_per_pic} MBs")


if __name__ == "__main__":
    main()

"""End-to-end (host-buffer, PCIe-inclusive) rates of the decode path, next to the device rate.

    python tools/e2e_bench.py [--gops 16] [--config c2] [--threads N]

Stages timed on one stream (seed 1729):
  parse     host VLC/record emitter (mp2vg_parse_es, multithreaded), .m2v bytes -> records
  upload    mp2vg_batch_upload: validation + level planning + pinned H2D copy of the records
  decode    device span of mp2vg_batch_decode (records resident in HBM; the bench's `value`)
  download  D2H of every decoded frame into host planes (frame_c layout)
  dropin    mp2v_decoder_c.decode(): parse + chunked upload/decode/download + display-order
            render callbacks, i.e. what a caller of the reference API sees
  reference (--ref) the real reference decoder on the same stream and host (bench.cpu_baseline)
Prints one JSON line.  DESIGN.md quotes these as the PCIe-inclusive rates (never `value`).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402
from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gops", type=int, default=16)
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--ref", action="store_true", help="also time the real reference (oracle/_ref/ref_decode) "
                    "on the same stream and host")
    ap.add_argument("--device-frames", action="store_true", help="drop-in with MP2VG_DECODER_DEVICE_FRAMES "
                    "(frames handed over in HBM, no D2H)")
    a = ap.parse_args()
    w, h, cf, extra, desc = bench.CONFIGS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=a.gops, seed=1729, **extra)

    t = time.perf_counter()
    p = R.Parsed(es, w, h, cf, threads=a.threads)
    t_parse = time.perf_counter() - t
    rec_bytes = p.pics.nbytes + p.mbs.nbytes + p.coefs.nbytes

    with R.DeviceContext(w, h, cf, slots=p.npics) as ctx:
        ctx.upload(p.pics, p.mbs, p.coefs)  # warm (allocations)
        t = time.perf_counter()
        ctx.upload(p.pics, p.mbs, p.coefs)
        t_up = time.perf_counter() - t
        ctx.decode()
        ctx.synchronize()
        dev = []
        for _ in range(5):
            ctx.decode()
            dev.append(ctx.batch_time_ms())
        t_dev = float(np.median(dev)) / 1000.0
        t = time.perf_counter()
        frames = [ctx.download(i) for i in range(p.npics)]
        t_down = time.perf_counter() - t
        frame_bytes = sum(x.nbytes for x in frames[0])

    count = [0]

    def render(frame):
        count[0] += 1

    cfg = decoder_config_t(w, h, cf, pictures_pool_size=24, num_threads=a.threads, device_frames=a.device_frames)
    dec = mp2v_decoder_c(cfg, render)
    t = time.perf_counter()
    dec.decode(es, len(es))
    t_drop = time.perf_counter() - t
    dec.close()
    assert count[0] == p.npics

    n = p.npics
    out = {
        "workload": f"{desc}, {a.gops} GOPs ({n} frames), seed 1729",
        "host_threads": a.threads,
        "parse_fps": round(n / t_parse, 1),
        "upload_GBps": round(rec_bytes / t_up / 1e9, 2), "upload_fps": round(n / t_up, 1),
        "record_bytes_per_frame": int(rec_bytes / n),
        "device_fps": round(n / t_dev, 1),
        "download_GBps": round(frame_bytes * n / t_down / 1e9, 2), "download_fps": round(n / t_down, 1),
        "dropin_fps": round(n / t_drop, 1), "dropin_device_frames": a.device_frames,
        "pcie_inclusive_fps": round(n / (t_up + t_dev + t_down), 1),
    }
    if a.ref:
        cb = bench.cpu_baseline(es, w, h, cf, n)
        out["reference_fps"] = cb["value"]
        out["reference_threads"] = cb["cores"]
        out["reference_fps_1thread"] = cb.get("value_1thread")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

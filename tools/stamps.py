"""Stage shares of the recon loop from the diagnostic stamp build (MP2VG_ABLATE=16; dev tool).

    tools/dev_build.sh
    MP2VG_LIB=tiny_mp2v_dec_amd/_var/dev/libmp2vg.so MP2VG_ABLATE=16 python tools/stamps.py [--gops 32] [--config c2]
Reads the per-mode s_memtime sums the stamp build adds into the pool pad (sink + 1024) and prints
each stage's share of the loop; quote shares only, never the stamp build's run time.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402
from tiny_mp2v_dec_amd._lib import lib  # noqa: E402

STAGES = ["wait taps + predict", "look-ahead issue", "dequant", "idct pass 1", "idct pass 2", "add/clip + store",
          "latch"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gops", type=int, default=32)
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    assert os.environ.get("MP2VG_ABLATE") == "16", "run with MP2VG_ABLATE=16"
    w, h, cf, extra, _ = bench.CONFIGS[a.config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=a.gops, seed=1729, **extra)
    p = R.Parsed(es, w, h, cf)
    hip = ctypes.CDLL("libamdhip64.so")
    with R.DeviceContext(w, h, cf, p.npics) as d:
        d.upload(p.pics, p.mbs, p.coefs)
        dp = ctypes.c_void_p()
        assert lib().mp2vg_sink_device_ptr(d.h, ctypes.byref(dp)) == 0
        addr = ctypes.c_void_p(dp.value + 2048 + 1024)  # geo.sink (kSinkOff) + 1024: the stamp sums
        assert hip.hipMemset(addr, 0, 3 * 8 * 8) == 0
        d.decode()
        d.synchronize()
        out = np.zeros(24, dtype=np.uint64)
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), addr, out.nbytes, 2) == 0
    for mcm, name in enumerate(["I", "P", "B"]):
        v = out[8 * mcm: 8 * mcm + 8].astype(np.float64)
        if v[7] == 0:
            continue
        tot = v[:7].sum()
        print(f"{name}: waves {int(v[7])}, cycles per wave {tot / v[7]:.0f}")
        for i, s in enumerate(STAGES):
            print(f"   {s:22s} {100 * v[i] / tot:5.1f} %   {v[i] / v[7]:8.0f} cycles/wave")


if __name__ == "__main__":
    main()

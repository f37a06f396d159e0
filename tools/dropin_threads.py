"""Drop-in end to end vs host thread count (dev tool, run on the GPU box): the c2 bench stream
decoded by mp2v_decoder_c with num_threads = T (parse workers = T - 1 since round 5, T - 2 when measured; decoder.cpp), host frames,
a null renderer; interleaved rounds, one JSON line per run.

    python tools/dropin_threads.py [gops] [threads...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402
from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c  # noqa: E402

gops = int(sys.argv[1]) if len(sys.argv) > 1 else 64
threads = [int(x) for x in sys.argv[2:]] or [16, 17, 18]
w, h, cf, extra, _ = bench.CONFIGS["c2"]
es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **extra)
for rnd in range(3):
    for t in threads:
        n = [0]
        dec = mp2v_decoder_c(decoder_config_t(w, h, cf, pictures_pool_size=24, num_threads=t),
                             lambda f: n.__setitem__(0, n[0] + 1))
        dec.decode(es)  # warm-up: pools, banks, streams
        n[0] = 0
        t0 = time.perf_counter()
        dec.decode(es)
        dt = time.perf_counter() - t0
        dec.close()
        print(json.dumps({"round": rnd, "num_threads": t, "parse_workers_then": t - 2, "frames": n[0],
                          "frames_per_s": round(n[0] / dt, 1)}), flush=True)

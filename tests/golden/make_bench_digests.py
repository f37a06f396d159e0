"""Expected per-frame digests of bench.py's timed batches, from the REAL reference decoder.

Run in the build container (needs oracle/_ref/ref_decode, built from /root/reference by
`make -C oracle ref`).  For every (config, GOPs, seed) that bench.py decodes by default -- one
stream per rank, seed 1729 + rank, ranks 0..7 for the multi-GPU configs -- the stream is
written exactly as bench.py writes it, decoded by the compiled reference at num_threads=1, and
each frame's digest (records.planes_digest, computed in ref_decode's render callback) is stored
in decode order, the order of bench.py's slots:
  tests/golden/bench_digests.npz   key "<config>_g<gops>_s<seed>" -> uint64[frames]
                                   key "digest_format" -> [DIGEST_FORMAT]
bench.py compares its device digests with these after the timed region and reports
"parity": "bit-exact" (or fails).  The reference's scheduler can render a stale pool slot
(see make_stream_fixtures.py), which shows as a repeated frame digest: such runs are retried.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = os.path.join(REPO, "oracle", "_ref", "ref_decode")

import bench  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

RANKS = 8
# the digest formula the entries were computed with (records.planes_digest): 1 = round 3's
# additive mix64(key) ^ d; 2 = mix64(mix64(key) ^ d), mixed after combining (round 4).  A file
# without this key, or with another value, is never resumed from or merged into.
DIGEST_FORMAT = bench.DIGEST_FORMAT
CASES = [("c1", 0)] + [("c2", s) for s in range(RANKS)] + [("c3", 0), ("c4", 0)] + [("c4", s) for s in range(1, RANKS)] + [("c5", 0)]
# (config, rank, GOPs): one-GOP c4 streams of all 8 ranks, for the 8-rank rehearsal of the c4
# scaling command (tests/test_bench_multirank.py: bench.py --gpus 8 --config c4 --gops 1)
CASES += [("c4", s, 1) for s in range(RANKS)]


def reference_digests(es, w, h, cf, tmp):
    path, dig = os.path.join(tmp, "s.m2v"), os.path.join(tmp, "s.dig")
    with open(path, "wb") as f:
        f.write(es)
    clean = []
    for _ in range(20):  # long 4K streams hit the reference's stale-slot race more often
        r = subprocess.run([REF, path, str(w), str(h), str(cf), "1", dig], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-400:])
        d = np.fromfile(dig, dtype="<u8")
        if len(set(d.tolist())) == len(d):  # no stale (repeated) frame
            clean.append(d)
            if len(clean) == 2:
                break
    if len(clean) < 2 or not np.array_equal(clean[0], clean[1]):
        raise RuntimeError("no two agreeing race-free reference runs")
    return clean[0]


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    only = set(sys.argv[1:])  # e.g. "c1" or "c4_g1": (re)compute only these cases, keep the other keys
    out = {}
    path = os.path.join(HERE, "bench_digests.npz")
    resume = bool(os.environ.get("MP2VG_DIGESTS_RESUME"))
    if (only or resume) and os.path.exists(path):
        with np.load(path) as d:
            fmt = int(d["digest_format"][0]) if "digest_format" in d.files else 1
            if fmt != DIGEST_FORMAT:
                if only:
                    sys.exit(f"{path} holds digest format {fmt}, not {DIGEST_FORMAT}: regenerate every config")
                print(f"{path}: digest format {fmt} != {DIGEST_FORMAT}, starting over")
            else:
                out = {k: d[k].copy() for k in d.files}
    out["digest_format"] = np.array([DIGEST_FORMAT], np.int64)
    with tempfile.TemporaryDirectory() as tmp:
        for case in CASES:
            config, rank = case[0], case[1]
            gops = case[2] if len(case) > 2 else bench.DEFAULT_GOPS[config]
            if only and config not in only and f"{config}_g{gops}" not in only:
                continue
            w, h, cf, gparams, _ = bench.CONFIGS[config]
            seed = 1729 + rank
            if resume and f"{config}_g{gops}_s{seed}" in out:
                continue  # resuming an interrupted run: keep the finished cases
            es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=seed, **gparams)
            parsed = R.Parsed(es, w, h, cf, threads=8)
            disp = reference_digests(es, w, h, cf, tmp)
            assert len(disp) == parsed.npics
            dec = np.zeros(parsed.npics, np.uint64)
            dec[parsed.display] = disp  # display position j holds decode index display[j]
            out[f"{config}_g{gops}_s{seed}"] = dec
            print(f"{config} g{gops} seed {seed}: {parsed.npics} frames")
            np.savez_compressed(path, **out)  # keep each finished case
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    main()

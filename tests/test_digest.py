"""The frame digest (records.planes_digest, the device digest_kernel and oracle/_ref/ref_decode's
render-callback digest are twins) must not cancel small paired errors: bench.py's parity claim
for every timed frame rests on it.

An additive digest sum(mix64(key) ^ d) moves by +-2^b when bit b of one dword flips, the sign
set by the key's bit, so two LSB errors of opposite sign in one byte lane cancel.  The digest
mixes after combining, sum(mix64(mix64(key) ^ d)), so each term is a pseudo-random function of
its dword.  These tests build exactly such a cancelling pair and check that the digest moves,
and that the compiled reference's digest equals the host twin on a real decode."""
import os
import subprocess

import numpy as np
import pytest

from tiny_mp2v_dec_amd import records as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref", "ref_decode")


def additive_digest(planes):
    """The round-3 (weak) digest, kept here only to show the cancelling pair is real."""
    total = np.uint64(0)
    row0 = 0
    with np.errstate(over="ignore"):
        for p in planes:
            p = np.ascontiguousarray(p)
            h, w = p.shape
            d = p.view("<u4").astype(np.uint64)
            rows = (np.arange(h, dtype=np.uint64) + np.uint64(row0))[:, None]
            xs = (np.arange(w // 4, dtype=np.uint64) * np.uint64(4))[None, :]
            total = total + np.sum(R._mix64((rows << np.uint64(32)) | xs) ^ d, dtype=np.uint64)
            row0 += h
    return int(total)


def cancelling_pair(planes):
    """Two byte-0 LSB flips in Y row 0 (dwords at x0, x1) that leave the additive digest
    unchanged: the key-xor-value bit 0 differs between the two positions."""
    y = planes[0]
    keys = R._mix64(np.arange(y.shape[1] // 4, dtype=np.uint64) * np.uint64(4))
    bit = (keys ^ y[0].view("<u4").astype(np.uint64)) & np.uint64(1)
    x0 = 0
    for j in range(1, len(bit)):
        if bit[j] != bit[x0]:
            return 0, 4 * j
    raise AssertionError("no cancelling pair in row 0")


def flipped(planes, x0, x1):
    out = [p.copy() for p in planes]
    out[0][0, x0] ^= 1
    out[0][0, x1] ^= 1
    return out


def test_digest_catches_a_pair_the_additive_digest_cancels():
    rng = np.random.default_rng(5)
    for _ in range(20):
        planes = [rng.integers(0, 256, (16, 32), np.uint8), rng.integers(0, 256, (8, 16), np.uint8),
                  rng.integers(0, 256, (8, 16), np.uint8)]
        x0, x1 = cancelling_pair(planes)
        bad = flipped(planes, x0, x1)
        assert additive_digest(bad) == additive_digest(planes)  # the weakness is real
        assert R.planes_digest(bad) != R.planes_digest(planes)


def test_digest_moves_for_every_single_lsb_and_sparse_pm1_pattern():
    rng = np.random.default_rng(6)
    planes = [rng.integers(0, 256, (16, 32), np.uint8), rng.integers(0, 256, (8, 16), np.uint8),
              rng.integers(0, 256, (8, 16), np.uint8)]
    base = R.planes_digest(planes)
    seen = {base}
    for p in range(3):
        for idx in range(planes[p].size):
            bad = [q.copy() for q in planes]
            bad[p].flat[idx] ^= 1
            seen.add(R.planes_digest(bad))
    assert len(seen) == 1 + sum(q.size for q in planes)  # all distinct
    for _ in range(200):  # sparse +-1 errors, 2-8 pixels
        bad = [q.copy() for q in planes]
        n = int(rng.integers(2, 9))
        for _ in range(n):
            p = int(rng.integers(0, 3))
            i = int(rng.integers(0, bad[p].size))
            v = int(bad[p].flat[i])
            bad[p].flat[i] = v + 1 if v < 255 else v - 1
        if any(not np.array_equal(a, b) for a, b in zip(bad, planes)):
            assert R.planes_digest(bad) != base


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref/ref_decode not built")
def test_reference_render_digest_is_the_host_twin(tmp_path):
    """ref_decode's per-frame digests (what tests/golden/bench_digests.npz holds) == planes_digest
    of the reference's own YUV output of the same stream."""
    w, h, cf = 176, 144, 1
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=1, gop_n=12, gop_m=3, seed=77)
    m2v = tmp_path / "s.m2v"
    m2v.write_bytes(es)
    dig, yuv = tmp_path / "s.dig", tmp_path / "s.yuv"
    fb = w * h + 2 * (w // 2) * (h // 2)
    # The reference's scheduler can render a stale pool slot under host load (its
    # multi-threaded path is racy; make_bench_digests.py retries for the same reason), so the pair
    # of runs (digest, YUV) is repeated until one pair agrees frame for frame: a race in either run
    # shows as a mismatch, a wrong digest function as a mismatch in every pair.
    def host_twins(frames):
        out = []
        for f in frames:
            out.append(R.planes_digest([f[:w * h].reshape(h, w), f[w * h:w * h + fb // 6].reshape(h // 2, w // 2),
                                        f[w * h + fb // 6:].reshape(h // 2, w // 2)]))
        return out

    for _ in range(10):
        for out in (dig, yuv):
            r = subprocess.run([REF, str(m2v), str(w), str(h), str(cf), "1", str(out)], capture_output=True,
                               text=True, timeout=120)
            assert r.returncode == 0, r.stderr[-300:]
        d = np.fromfile(dig, dtype="<u8")
        raw = np.fromfile(yuv, dtype=np.uint8)
        assert len(raw) == fb * len(d) and len(d) == 12
        twins = host_twins([raw[k * fb:(k + 1) * fb] for k in range(len(d))])
        if [int(x) for x in d] == [int(x) for x in twins]:
            break
    assert [int(x) for x in d] == [int(x) for x in twins]

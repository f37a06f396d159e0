"""Shared test helpers: oracle-vs-golden plumbing (oracle = checker only)."""
import hashlib

import numpy as np

import _oracle
from tiny_mp2v_dec_amd.records import Parsed


def oracle_frames(parsed: Parsed):
    """Decode-order frames from the C oracle: list of [Y, U, V] arrays."""
    g, pool = _oracle.reconstruct(parsed.width, parsed.height, parsed.chroma_format, parsed.pics, parsed.mbs,
                                  parsed.coefs, parsed.npics)
    frames = []
    for d in range(parsed.npics):
        base = d * g.slot_bytes
        planes = []
        for p in range(3):
            st, pw, ph = g.stride[p], g.pw[p], g.ph[p]
            arr = pool[base + g.plane_off[p]: base + g.plane_off[p] + st * ph].reshape(ph, st)[:, :pw]
            planes.append(arr.copy())
        frames.append(planes)
    return frames


def yuv_md5(planes):
    h = hashlib.md5()
    for p in planes:
        h.update(np.ascontiguousarray(p).tobytes())
    return h.hexdigest()

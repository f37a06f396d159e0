"""CPU: the pass-1 IDCT folds of recon.hip (idct_1d<true>) equal the exact SSE2 transform
(idct_sse2.hpp:23-65, ref) whenever inputs 1-7 lie in the dequant clamp range [-2048, 2047]
(mb_decoder.cpp:146) and input 0 (QFS[0]: intra DC or the unclamped '1s' coefficient) is any int16.

The model below is plain int64 numpy with explicit int16 wrap (slli) and saturation
(adds/subs); every folded product is asserted to stay below 2^31 (the kernel multiplies in 32 bits).
"""
import itertools

import numpy as np


def _sat(x):
    return np.clip(x, -32768, 32767)


def _wrap(x):
    return ((x + 32768) % 65536) - 32768


def _adds(a, b):
    return _sat(a + b)


def _subs(a, b):
    return _sat(a - b)


def _shl(a, n):
    return _wrap(a << n)


def _mulhi(a, c):
    assert np.abs(a * c).max() < 2 ** 31
    return _wrap((a * c) >> 16)


def _mulhi_x2(a, c):  # slli(mulhi(a, c), 1) as the kernel computes it: high half of a*2c, bit 0 cleared
    assert np.abs(a * 2 * c).max() < 2 ** 31
    return _wrap(((a * 2 * c) >> 16) & ~1)


def idct_1d(s, p1):
    s = [np.asarray(x, dtype=np.int64) for x in s]
    v15 = _adds(_mulhi_x2(s[0], 27145), _shl(s[0], 1))
    v26 = _mulhi(s[1], -5037 + 262144) if p1 else _adds(_mulhi(s[1], -5037), _shl(s[1], 2))
    v21 = _mulhi(s[2], -19954 + 262144) if p1 else _adds(_mulhi(s[2], -19954), _shl(s[2], 2))
    v28 = _mulhi_x2(s[3], -22089 + 131072) if p1 else _adds(_mulhi_x2(s[3], -22089), _shl(s[3], 2))
    v16 = _mulhi_x2(s[4], 27145 + 65536) if p1 else _adds(_mulhi_x2(s[4], 27145), _shl(s[4], 1))
    v25 = _mulhi(s[5], 14567 + 131072) if p1 else _adds(_mulhi(s[5], 14567), _shl(s[5], 1))
    v22 = _adds(_mulhi_x2(s[6], 17391), s[6])
    v27 = _mulhi_x2(s[7], 25570)
    v19, v20 = _subs(v25, v28), _subs(v26, v27)
    v23, v24 = _adds(v26, v27), _adds(v25, v28)
    v7, v11 = _adds(v23, v24), _adds(v21, v22)
    v13, v17 = _subs(v23, v24), _subs(v21, v22)
    v8, v9 = _adds(v15, v16), _subs(v15, v16)
    v18 = _mulhi(_subs(v19, v20), 25079)
    v12 = _subs(v18, _mulhi(v19, 20090 + 65536) if p1 else _adds(v19, _mulhi(v19, 20090)))
    v14 = _subs(_subs(v20, _mulhi(v20, 30068)), v18)
    v6 = _subs(_shl(v14, 1), v7)
    v5 = _subs(_mulhi(v13, 27145 + 65536) if p1 else _adds(v13, _mulhi(v13, 27145)), v6)
    v4 = _adds(v5, _shl(v12, 1))
    v10 = _subs(_mulhi(v17, 27145 + 65536) if p1 else _adds(v17, _mulhi(v17, 27145)), v11)
    v0, v1, v2, v3 = _adds(v8, v11), _adds(v9, v10), _subs(v9, v10), _subs(v8, v11)
    return np.stack([_adds(v0, v7), _adds(v1, v6), _adds(v2, v5), _subs(v3, v4),
                     _adds(v3, v4), _subs(v2, v5), _subs(v1, v6), _subs(v0, v7)])


def test_pass1_folds_equal_exact_transform_random():
    rng = np.random.default_rng(7)
    n = 1_000_000
    s = [rng.integers(-32768, 32768, n)] + [rng.integers(-2048, 2048, n) for _ in range(7)]
    assert np.array_equal(idct_1d(s, False), idct_1d(s, True))
    edge = np.array([-2048, -2047, -1, 0, 1, 2046, 2047])
    s = [rng.integers(-32768, 32768, n)] + [rng.choice(edge, n) for _ in range(7)]
    assert np.array_equal(idct_1d(s, False), idct_1d(s, True))


def test_pass1_folds_equal_exact_transform_corners():
    corners = np.array(list(itertools.product([-2048, 2047], repeat=7))).T
    s0 = np.repeat(np.arange(-32768, 32768, 97), corners.shape[1])
    c = np.tile(corners, (1, len(s0) // corners.shape[1]))
    out = idct_1d([s0] + list(c), False)
    assert np.array_equal(out, idct_1d([s0] + list(c), True))
    assert (np.abs(out) == 32767).any() or (out == -32768).any()  # the exact model does saturate here


"""Generate per-kernel golden vectors from the REAL reference kernels.

Run in the build container (needs oracle/_ref/ref_kernels, built by `make -C oracle ref` from
/root/reference).  Inputs are seeded (1729, the reference tests' seed: test/gtest/simd/
mc_test.cpp:20-25, idct_test.cpp:53-57); the outputs are produced by the reference's own
x86 kernels:
  idct: inverse_dct_template<false/true> (idct_sse2.hpp:96-120)
  mc:   mc_pred_{16,8}xh / mc_bidir_{16,8}xh tables (mc.cpp:4-25 -> mc_sse2.hpp)
and committed as tests/golden/idct_vectors.npz / mc_vectors.npz.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_KERNELS = os.path.join(REPO, "oracle", "_ref", "ref_kernels")


def idct_inputs(rng):
    blocks = []
    # 1) the reference test's distribution: uniform [0,255] coefficients (idct_test.cpp:53-57)
    blocks.append(rng.integers(0, 256, size=(400, 64)))
    # 2) sparse dequantised-like blocks, |v| <= 300 (no saturation)
    b = np.zeros((800, 64), np.int64)
    for k in range(len(b)):
        n = rng.integers(1, 10)
        pos = rng.choice(64, n, replace=False)
        b[k, pos] = rng.integers(-300, 301, size=n)
    blocks.append(b)
    # 3) high-amplitude blocks (+-2047 / -2048 class): saturation fires here
    b = np.zeros((800, 64), np.int64)
    for k in range(len(b)):
        n = rng.integers(1, 64)
        pos = rng.choice(64, n, replace=False)
        b[k, pos] = rng.integers(-2048, 2048, size=n)
    blocks.append(b)
    # 4) DC-only and single-coefficient blocks at the extremes
    b = np.zeros((128, 64), np.int64)
    for k in range(64):
        b[k, k] = 2047 if k % 2 == 0 else -2048
    for k in range(64, 128):
        b[k, 0] = (k - 64) * 64 - 2048
    blocks.append(b)
    F = np.concatenate(blocks).astype(np.int16)
    pred = rng.integers(0, 256, size=(F.shape[0], 64)).astype(np.uint8)
    return F, pred


def run_idct(F, pred, tmp):
    rec = np.zeros(F.shape[0], dtype=[("F", "<i2", 64), ("pred", "u1", 64)])
    rec["F"] = F
    rec["pred"] = pred
    fin, fout = os.path.join(tmp, "idct.in"), os.path.join(tmp, "idct.out")
    rec.tofile(fin)
    subprocess.check_call([REF_KERNELS, "idct", fin, fout])
    out = np.fromfile(fout, dtype=np.uint8).reshape(F.shape[0], 2, 64)
    return out[:, 0], out[:, 1]


def mc_inputs(rng):
    stride, rows = 64, 48
    A = rng.integers(0, 256, size=stride * rows).astype(np.uint8)
    B = rng.integers(0, 256, size=stride * rows).astype(np.uint8)
    cases = []
    for bidir, nidx in ((0, 4), (1, 16)):
        for width in (16, 8):
            for height in ((8, 16) if width == 16 else (4, 8, 16)):
                for idx in range(nidx):
                    for _ in range(6):
                        offa = int(rng.integers(0, 8)) * stride + int(rng.integers(0, stride - width - 1))
                        offb = int(rng.integers(0, 8)) * stride + int(rng.integers(0, stride - width - 1))
                        if width == 16:  # the SSE2 16-wide store is aligned (mc_sse2.hpp:45)
                            pass
                        cases.append((bidir, width, height, idx, offa, offb, 0, 0))
    return stride, rows, A, B, np.array(cases, dtype=np.int32)


def run_mc(stride, rows, A, B, cases, tmp):
    fin, fout = os.path.join(tmp, "mc.in"), os.path.join(tmp, "mc.out")
    with open(fin, "wb") as f:
        f.write(np.array([stride, rows, len(cases), 0], np.int32).tobytes())
        f.write(A.tobytes())
        f.write(B.tobytes())
        f.write(cases.tobytes())
    subprocess.check_call([REF_KERNELS, "mc", fin, fout])
    return np.fromfile(fout, dtype=np.uint8)


def main():
    if not os.path.exists(REF_KERNELS):
        sys.exit("build the reference first: make -C oracle ref")
    rng = np.random.default_rng(1729)
    with tempfile.TemporaryDirectory() as tmp:
        F, pred = idct_inputs(rng)
        put, add = run_idct(F, pred, tmp)
        np.savez_compressed(os.path.join(HERE, "idct_vectors.npz"), F=F, pred=pred, put=put, add=add)
        stride, rows, A, B, cases = mc_inputs(rng)
        out = run_mc(stride, rows, A, B, cases, tmp)
        np.savez_compressed(os.path.join(HERE, "mc_vectors.npz"), stride=stride, rows=rows, A=A, B=B,
                            cases=cases, out=out)
    print("idct blocks", F.shape[0], "mc cases", len(cases))


if __name__ == "__main__":
    main()

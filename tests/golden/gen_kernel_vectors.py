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


def idct_wide(F):
    """The SSE2 flow graph of idct_sse2.hpp:23-120 evaluated in int64 with NO 16-bit saturation or
    wrap-around: where its output differs from the reference's, saturation fired in that block."""
    F = F.astype(np.int64).reshape(-1, 8, 8)

    def mulhi(a, c):
        return (a * c) >> 16

    def pass1d(s):  # s[..., i, j]: transform over i for every column j
        s = [s[:, i, :] for i in range(8)]
        v15 = (mulhi(s[0], 27145) << 1) + (s[0] << 1)
        v26 = mulhi(s[1], -5037) + (s[1] << 2)
        v21 = mulhi(s[2], -19954) + (s[2] << 2)
        v28 = (mulhi(s[3], -22089) << 1) + (s[3] << 2)
        v16 = (mulhi(s[4], 27145) << 1) + (s[4] << 1)
        v25 = mulhi(s[5], 14567) + (s[5] << 1)
        v22 = (mulhi(s[6], 17391) << 1) + s[6]
        v27 = mulhi(s[7], 25570) << 1
        v19, v20, v23, v24 = v25 - v28, v26 - v27, v26 + v27, v25 + v28
        v7, v11, v13, v17 = v23 + v24, v21 + v22, v23 - v24, v21 - v22
        v8, v9 = v15 + v16, v15 - v16
        v18 = mulhi(v19 - v20, 25079)
        v12 = v18 - (v19 + mulhi(v19, 20090))
        v14 = (v20 - mulhi(v20, 30068)) - v18
        v6 = (v14 << 1) - v7
        v5 = (v13 + mulhi(v13, 27145)) - v6
        v4 = v5 + (v12 << 1)
        v10 = (v17 + mulhi(v17, 27145)) - v11
        v0, v1, v2, v3 = v8 + v11, v9 + v10, v9 - v10, v8 - v11
        out = [v0 + v7, v1 + v6, v2 + v5, v3 - v4, v3 + v4, v2 - v5, v1 - v6, v0 - v7]
        return np.stack(out, axis=1)

    b = pass1d(F)
    b = pass1d(np.transpose(b, (0, 2, 1)))
    return np.clip(b >> 6, 0, 255).astype(np.uint8).reshape(-1, 64)


def chain_pairs(F, nblocks):
    """Blocks for the GPU run of the IDCT vectors (tests/test_gpu_parity.py): an I picture whose
    blocks are put-vectors and a P picture (zero MV) whose blocks add add-vectors onto them.  The
    record path applies mismatch control (mb_decoder.cpp:150-152): it is a no-op exactly when
    the coefficient sum is odd (intra: DC excluded), so only such vectors are used."""
    s_ac = F[:, 1:].astype(np.int64).sum(1)
    s_all = F.astype(np.int64).sum(1)
    put_sel = np.nonzero(s_ac % 2 == 1)[0]
    add_sel = np.nonzero(s_all % 2 == 1)[0]
    j = np.arange(nblocks)
    return put_sel[j % len(put_sel)], add_sel[(j * 7 + 3) % len(add_sel)]


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
        # chain: reference add of add-vector a over the put output of put-vector p (the GPU test's
        # P picture predicts from the I picture with a zero MV); 16x12 MBs x 6 blocks (4:2:0)
        pidx, aidx = chain_pairs(F, 16 * 12 * 6)
        _, chain_add = run_idct(F[aidx], put[pidx], tmp)
        wide = idct_wide(F)
        sat = np.any(wide != put, axis=1)  # saturation / wrap changed the reference's put output
        np.savez_compressed(os.path.join(HERE, "idct_chain.npz"), put_idx=pidx, add_idx=aidx, add=chain_add,
                            put_saturates=sat[pidx])
        stride, rows, A, B, cases = mc_inputs(rng)
        out = run_mc(stride, rows, A, B, cases, tmp)
        np.savez_compressed(os.path.join(HERE, "mc_vectors.npz"), stride=stride, rows=rows, A=A, B=B,
                            cases=cases, out=out)
    print("idct blocks", F.shape[0], "mc cases", len(cases))


if __name__ == "__main__":
    main()

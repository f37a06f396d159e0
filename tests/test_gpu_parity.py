"""GPU parity: the HIP reconstruct path (through the C ABI) against the reference's golden output
and against the C oracle.  Bit-exact everywhere (integer/byte work)."""
import numpy as np
import pytest

from conftest import load_manifest, read_stream
from helpers import oracle_frames, yuv_md5
from tiny_mp2v_dec_amd import records as R
from tiny_mp2v_dec_amd._lib import MB_BWD, MB_DCT_FIELD, MB_FIELD_MC, MB_FWD, MB_INTRA, COEF_DC, COEF_FIRST1S

pytestmark = pytest.mark.gpu

MANIFEST = load_manifest()


def gpu_decode(parsed, device=0):
    with R.DeviceContext(parsed.width, parsed.height, parsed.chroma_format, slots=parsed.npics, device=device) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        return [ctx.download(int(p["dst_slot"])) for p in parsed.pics]


@pytest.mark.parametrize("entry", MANIFEST, ids=[e["name"] for e in MANIFEST])
def test_golden_streams_bit_exact(entry):
    """Whole streams: GPU frames in display order == the compiled reference's YUV (per-frame MD5)."""
    parsed = R.Parsed(read_stream(entry), entry["width"], entry["height"], entry["chroma_format"])
    frames = gpu_decode(parsed)
    got = [yuv_md5(frames[d]) for d in parsed.display]
    assert got == entry["md5"]


def random_batch(width, height, cf, npics, seed, field=True, big=False, n_intra=1):
    """Synthetic record batch exercising every record feature (random MVs kept inside the planes):
    pictures 0..n_intra-1 are I, the next one P (forward from the one before), the rest B (forward
    p-1, backward p-2)."""
    rng = np.random.default_rng(seed)
    mbw, mbh = width // 16, height // 16
    nb = {1: 6, 2: 8, 3: 12}[cf]
    n = mbw * mbh
    pics = np.zeros(npics, R.PIC_DTYPE)
    mbs = np.zeros(n * npics, R.MB_DTYPE)
    coefs = []
    cw, ch = (16 if cf == 3 else 8), (8 if cf == 1 else 16)
    for p in range(npics):
        pics[p]["dst_slot"] = p
        pics[p]["fwd_slot"] = p - 1 if p >= n_intra else -1
        pics[p]["bwd_slot"] = p - 2 if p >= n_intra + 1 else -1
        pics[p]["picture_coding_type"] = 1 if p < n_intra else (2 if p == n_intra else 3)
        pics[p]["mb_first"] = p * n
        pics[p]["mb_width"], pics[p]["mb_height"] = mbw, mbh
        pics[p]["alternate_scan"] = rng.integers(0, 2)
        pics[p]["W"] = rng.integers(1, 256 if big else 48, size=(4, 64))
        for k in range(n):
            m = mbs[p * n + k]
            m["x"], m["y"] = k % mbw, k // mbw
            m["qscale"] = rng.integers(1, 113)
            intra = p < n_intra or rng.random() < 0.1
            flags = 0
            if intra:
                flags |= MB_INTRA
                cbp = (1 << nb) - 1
            else:
                d = rng.integers(0, 3) if p > n_intra else 0
                flags |= [MB_FWD, MB_BWD, MB_FWD | MB_BWD][d]
                fld = field and rng.random() < 0.3
                if fld:
                    flags |= MB_FIELD_MC
                    for r in range(2):
                        for s in range(2):
                            if rng.random() < 0.5:
                                flags |= 1 << (8 + 2 * r + s)
                # vectors that keep every read inside every plane
                for r in range(2 if fld else 1):
                    for s in range(2):
                        for _ in range(20):
                            mx, my = rng.integers(-40, 40), rng.integers(-40, 40)
                            if _inside(width, height, cf, m["x"], m["y"], mx, my, fld, (flags >> (8 + 2 * r + s)) & 1):
                                break
                        else:
                            mx, my = 0, 0
                            if fld:
                                flags &= ~(1 << (8 + 2 * r + s))
                                flags |= r << (8 + 2 * r + s)
                        m["mv"][r, s] = (mx, my)
                cbp = int(rng.integers(0, 1 << nb)) if rng.random() < 0.7 else 0
            if cbp and rng.random() < 0.4 and cf != 3:  # 4:4:4 field DCT is refused (test_validate.py)
                flags |= MB_DCT_FIELD
            m["flags"], m["cbp"] = flags, cbp
            m["coef_off"] = len(coefs)
            for b in range(nb):
                if not cbp >> b & 1:
                    continue
                pos = 0
                if intra:
                    coefs.append(R._lib.coef_pack(int(rng.integers(0, 2048)), 0, b, COEF_DC, m["x"]))
                    pos = 1
                elif rng.random() < 0.3:
                    coefs.append(R._lib.coef_pack(int(rng.choice([-1, 1])), 0, b, COEF_FIRST1S, m["x"]))
                    pos = 1
                ncoef = int(rng.integers(0 if intra else 1, 20))
                for _ in range(ncoef):
                    pos += int(rng.integers(0, 4))
                    if pos > 63:
                        break
                    lvl = int(rng.integers(-2048, 2048)) if (big and rng.random() < 0.3) else int(rng.integers(-40, 41))
                    coefs.append(R._lib.coef_pack(lvl, pos, b, 0, m["x"]))
                    pos += 1
            m["ncoef"] = len(coefs) - m["coef_off"]
    return pics, mbs, np.array(coefs, dtype=np.uint32)


def _inside(width, height, cf, mbx, mby, mvx, mvy, field, fs):
    pw = [width] + [width if cf == 3 else width // 2] * 2
    ph = [height] + [height if cf != 1 else height // 2] * 2
    for plane in range(3):
        mx, my = mvx, mvy
        if plane:
            if cf < 3:
                mx >>= 1
            if cf < 2:
                my >>= 1
        w = 16 if plane == 0 else (16 if cf == 3 else 8)
        h = 16 if plane == 0 else (8 if cf == 1 else 16)
        x0 = mbx * w + (mx >> 1)
        x1 = x0 + w - 1 + (mx & 1)
        if not field:
            y0 = mby * h + (my >> 1)
            y1 = y0 + h - 1 + (my & 1)
        else:
            y0 = mby * h + fs + 2 * (my >> 1)
            y1 = y0 + 2 * (h // 2 - 1) + 2 * (my & 1)
        if x0 < 0 or y0 < 0 or x1 > pw[plane] - 1 or y1 > ph[plane] - 1:
            return False
    return True


class _P:  # minimal Parsed-like holder for oracle_frames
    def __init__(self, w, h, cf, pics, mbs, coefs):
        self.width, self.height, self.chroma_format = w, h, cf
        self.pics, self.mbs, self.coefs = pics, mbs, coefs
        self.npics = len(pics)


@pytest.mark.parametrize("cf", [1, 2, 3])
@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("size", [(96, 64), (128, 48)], ids=["6mb_rows", "8mb_rows"])
def test_random_records_vs_oracle(cf, big, size):
    """Synthetic record batches (all MB kinds, field MC / DCT, saturating levels) vs the oracle.
    8-MB rows (a multiple of the kernel's 4-MB group): the P/B launches' workgroups take two
    one-row slices each (runtime.cpp plan_batch `mates`); a launch of one picture's three rows
    leaves a workgroup with one slice."""
    w, h = size
    pics, mbs, coefs = random_batch(w, h, cf, 5, seed=1729 + cf + 10 * big, big=big)
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    got = gpu_decode(_P(w, h, cf, pics, mbs, coefs))
    for p in range(len(pics)):
        for k in range(3):
            assert np.array_equal(got[p][k], exp[p][k]), (p, k)


@pytest.mark.parametrize("cf", [1, 2, 3])
def test_anchor_tiles_across_batches(cf):
    """The taps read references from the anchor tiles (recon.hip tile_off) that I and P pictures
    store.  Records may also use B pictures as references (never in an MPEG-2 stream): their tiles
    are rebuilt from the frame, inside a batch right after the B picture's launch, and across
    batches when a batch reads a slot whose last writer stored none (runtime.cpp TilePlan).  Two
    batches, pictures 0-2 then 3-4: picture 3 reads B picture 2 of the first batch, picture 4
    reads B pictures 3 and 2; every frame vs the oracle."""
    w, h = 96, 64
    pics, mbs, coefs = random_batch(w, h, cf, 5, seed=4242 + cf)
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    n = (w // 16) * (h // 16)
    c0 = int(mbs["coef_off"][3 * n])
    p2 = pics[3:].copy()
    p2["mb_first"] -= 3 * n
    m2 = mbs[3 * n:].copy()
    m2["coef_off"] -= c0
    with R.DeviceContext(w, h, cf, slots=5) as ctx:
        ctx.upload(pics[:3], mbs[:3 * n], coefs[:c0])
        ctx.decode()
        ctx.upload(p2, m2, coefs[c0:])
        ctx.decode()
        ctx.synchronize()
        for p in range(5):
            got = ctx.download(p)
            for k in range(3):
                assert np.array_equal(got[k], exp[p][k]), (p, k)


@pytest.mark.parametrize("cf", [1, 2, 3])
def test_one_direction_b_pictures_through_the_p_loop(cf):
    """B pictures that predict in one direction only (a closed GOP's leading B pictures: backward
    only) run the one-reference P loop with that reference, its vectors and field selects
    (runtime.cpp plan_batch, recon.hip issue_pass): in a P launch (picture 2, backward only, beside
    P picture 1) and inside a mixed launch (picture 5, backward only, beside two-direction picture
    4); picture 3 is forward only.  Every frame vs the oracle."""
    w, h = 96, 64
    pics, mbs, coefs = random_batch(w, h, cf, 6, seed=9090 + cf)
    n = (w // 16) * (h // 16)
    for p, keep in ((2, MB_BWD), (3, MB_FWD), (5, MB_BWD)):
        m = mbs[p * n:(p + 1) * n]
        inter = (m["flags"] & MB_INTRA) == 0
        m["flags"][inter] = (m["flags"][inter] & np.uint16(0xFFFF & ~(MB_FWD | MB_BWD))) | keep
    of_pic, modes = R.plan_batch(w, h, cf, 6, pics, mbs, coefs, one_stream=True)
    assert modes[of_pic[1]] == 1 and of_pic[2] == of_pic[1]  # P + backward-only B: a P launch
    assert modes[of_pic[5]] == 3 and of_pic[4] == of_pic[5]  # one- and two-direction B: mixed
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    got = gpu_decode(_P(w, h, cf, pics, mbs, coefs))
    for p in range(len(pics)):
        for k in range(3):
            assert np.array_equal(got[p][k], exp[p][k]), (p, k)


@pytest.mark.parametrize("cf", [1, 2, 3])
def test_i_only_batch_then_predictions(cf):
    """An I-only batch in which few pictures store anchor tiles (the last two, which a later batch
    may read; runtime.cpp plan_batch / TilePlan) stores exactly those pictures' tiles from the I
    kernel (mode 0; the tile-free mode 4 is a dev switch).  Batch 1: 12 I pictures; batch 2: a P
    picture predicting from picture 11 and B pictures from pictures 11 and 10, read through the
    tiles; every frame vs the oracle."""
    w, h = 96, 64
    pics, mbs, coefs = random_batch(w, h, cf, 16, seed=5150 + cf, n_intra=12)
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    n = (w // 16) * (h // 16)
    c0 = int(mbs["coef_off"][12 * n])
    assert set(R.plan_batch(w, h, cf, 16, pics[:12], mbs[:12 * n], coefs[:c0])[1].tolist()) == {0}
    p2 = pics[12:].copy()
    p2["mb_first"] -= 12 * n
    m2 = mbs[12 * n:].copy()
    m2["coef_off"] -= c0
    with R.DeviceContext(w, h, cf, slots=16) as ctx:
        ctx.upload(pics[:12], mbs[:12 * n], coefs[:c0])
        ctx.decode()
        ctx.upload(p2, m2, coefs[c0:])
        ctx.decode()
        ctx.synchronize()
        for p in range(16):
            got = ctx.download(p)
            for k in range(3):
                assert np.array_equal(got[k], exp[p][k]), (p, k)


def test_external_reference_write_then_invalidate():
    """A reference slot written from outside the decode (here a device-to-device copy of another
    context's decoded I picture through mp2vg_slot_device_ptr, as an RCCL receive would) is seen
    by later predictions only after mp2vg_invalidate_slot: the taps read the slot's anchor tiles,
    which the invalidated slot gets rebuilt from its frame before the next batch reads it."""
    import ctypes
    from tiny_mp2v_dec_amd import _lib
    from tiny_mp2v_dec_amd.decoder import _hip_lib
    w, h, cf = 96, 64, 1
    pics, mbs, coefs = random_batch(w, h, cf, 3, seed=777)
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    n = (w // 16) * (h // 16)
    c0 = int(mbs["coef_off"][n])
    rest, mrest = pics[1:].copy(), mbs[n:].copy()
    rest["mb_first"] -= n
    mrest["coef_off"] -= c0
    with R.DeviceContext(w, h, cf, slots=3) as src, R.DeviceContext(w, h, cf, slots=3) as dst:
        src.upload(pics[:1], mbs[:n], coefs[:c0])  # the I picture, decoded into src's slot 0
        src.decode()
        src.synchronize()
        ps, pd = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(_lib.lib().mp2vg_slot_device_ptr(src.h, 0, ctypes.byref(ps)), "slot_device_ptr")
        _lib.check(_lib.lib().mp2vg_slot_device_ptr(dst.h, 0, ctypes.byref(pd)), "slot_device_ptr")
        assert _hip_lib().hipMemcpy(pd.value, ps.value, int(src.slot_bytes), 3) == 0  # device to device
        _lib.check(_lib.lib().mp2vg_invalidate_slot(dst.h, 0), "invalidate_slot")
        with pytest.raises(_lib.Mp2vgError):
            _lib.check(_lib.lib().mp2vg_invalidate_slot(dst.h, 3), "invalidate_slot")
        dst.upload(rest, mrest, coefs[c0:])  # the P and B pictures predict from slot 0
        dst.decode()
        dst.synchronize()
        for p in range(3):
            got = dst.download(p)
            assert all(np.array_equal(got[k], exp[p][k]) for k in range(3)), p


def test_full_size_1080p_digest_vs_oracle():
    """BASELINE config size (1920x1088 4:2:0, one closed GOP of the §8d C2 mix): device digest of
    every frame == host digest of the oracle's frames (size-independent checksum-of-checksums)."""
    es = R.generate_es(width=1920, height=1088, chroma_format=1, n_gops=1, gop_n=12, gop_m=3, seed=99)
    parsed = R.Parsed(es, 1920, 1088, 1)
    exp = oracle_frames(parsed)
    with R.DeviceContext(1920, 1088, 1, slots=parsed.npics) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        dig = ctx.digests(np.arange(parsed.npics))
        for p in range(parsed.npics):  # every frame byte for byte, not only its digest
            got = ctx.download(p)
            assert all(np.array_equal(got[k], exp[p][k]) for k in range(3)), p
    assert len(dig) == 12
    assert [int(x) for x in dig] == [R.planes_digest(f) for f in exp]


def test_device_digest_catches_a_cancelling_lsb_pair():
    """Two complementary LSB flips in one byte lane of two dwords of a decoded slot (the pair an
    additive digest cancels, tests/test_digest.py) move the device digest, and the moved digest
    is the host twin's digest of the flipped planes."""
    import ctypes
    from test_digest import additive_digest, cancelling_pair, flipped
    from tiny_mp2v_dec_amd import _lib
    from tiny_mp2v_dec_amd.decoder import _hip_lib
    es = R.generate_es(width=176, height=144, chroma_format=1, n_gops=1, gop_n=12, gop_m=3, seed=31)
    parsed = R.Parsed(es, 176, 144, 1)
    with R.DeviceContext(176, 144, 1, slots=parsed.npics) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        slot = parsed.npics - 1
        planes = ctx.download(slot)
        before = int(ctx.digests(np.array([slot]))[0])
        assert before == R.planes_digest(planes)
        x0, x1 = cancelling_pair(planes)
        bad = flipped(planes, x0, x1)
        assert additive_digest(bad) == additive_digest(planes)
        ptr = ctypes.c_void_p()
        _lib.check(_lib.lib().mp2vg_slot_device_ptr(ctx.h, slot, ctypes.byref(ptr)), "slot_device_ptr")
        row = np.ascontiguousarray(bad[0][0])  # Y row 0 sits at the slot base (plane offset 0)
        assert _hip_lib().hipMemcpy(ptr.value, row.ctypes.data, row.nbytes, 1) == 0  # host to device
        after = int(ctx.digests(np.array([slot]))[0])
        assert np.array_equal(ctx.download(slot)[0], bad[0])
    assert after != before
    assert after == R.planes_digest(bad)


def test_back_to_back_batches_and_their_timing_events():
    """Batches decoded back to back without a host sync (as bench.py times them): a re-upload
    into the other record bank while decodes are queued leaves every frame bit-exact, and every
    batch's HIP events are readable afterwards (mp2vg_batch_times keeps the last 64)."""
    from tiny_mp2v_dec_amd.records import generate_es
    es_a = generate_es(width=176, height=144, chroma_format=1, n_gops=3, gop_n=12, gop_m=3, seed=61)
    es_b = generate_es(width=176, height=144, chroma_format=1, n_gops=3, gop_n=12, gop_m=3, seed=62)
    pa, pb = R.Parsed(es_a, 176, 144, 1), R.Parsed(es_b, 176, 144, 1)
    assert pa.npics == pb.npics
    with R.DeviceContext(176, 144, 1, slots=pa.npics) as ctx:
        ctx.upload(pa.pics, pa.mbs, pa.coefs)
        for _ in range(5):
            ctx.decode()
        ctx.upload(pb.pics, pb.mbs, pb.coefs)  # other bank; batch a's decodes may still be queued
        for _ in range(3):
            ctx.decode()
        ctx.synchronize()
        got = [yuv_md5(ctx.download(int(p["dst_slot"]))) for p in pb.pics]
        times = [ctx.batch_times(back) for back in range(8)]
        with pytest.raises(RuntimeError):
            ctx.batch_times(8)
    exp = [yuv_md5(f) for f in oracle_frames(pb)]
    assert got == exp
    for span, launches in times:
        assert span > 0 and launches and all(t > 0 for t in launches)


@pytest.mark.parametrize("config", ["c1", "c3", "c4", "c5"])
def test_bench_config_full_size_every_frame_vs_oracle(config):
    """The other bench configurations at full size (SURVEY §8d C1 1080p 4:2:0 I-only, C3 1080p
    4:2:2 IPB, C4 4K 4:2:0 IPB, C5 1080p 4:4:4 I-only high bitrate): one closed GOP (C1/C5: 4 I
    pictures) generated exactly
    as bench.py generates it, every frame's device digest == the digest of the oracle's frame,
    and the first and last frames compared byte for byte."""
    import importlib
    bench = importlib.import_module("bench")
    width, height, cf, gparams, _ = bench.CONFIGS[config]
    es = R.generate_es(width=width, height=height, chroma_format=cf, n_gops=4 if config in ("c1", "c5") else 1,
                       seed=1729, **gparams)
    parsed = R.Parsed(es, width, height, cf)
    exp = oracle_frames(parsed)
    with R.DeviceContext(width, height, cf, slots=parsed.npics) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        dig = ctx.digests(np.arange(parsed.npics))
        for p in (0, parsed.npics - 1):
            got = ctx.download(p)
            assert all(np.array_equal(got[k], exp[p][k]) for k in range(3)), (config, p)
    assert [int(x) for x in dig] == [R.planes_digest(f) for f in exp]


# ISO 13818-2 zig-zag scan (scan position -> raster index, row = vertical frequency); QFS is
# stored transposed (reference scan_c.cpp:4-21), so position i lands at QFS[col * 8 + row]
_ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
           13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
           45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
_QFS_OF_POS = [(r % 8) * 8 + r // 8 for r in _ZIGZAG]


def test_reference_idct_vectors_through_hip():
    """The reference's own SSE2 IDCT outputs (tests/golden/idct_chain.npz, from
    inverse_dct_template<false/true>, idct_sse2.hpp:96-120) reproduced by the HIP kernel.

    With every quantiser matrix entry 16 and quantiser_scale 1 the dequant is the identity
    (intra (|L|*16*1)>>4, non-intra ((2|L|+1)*16*1)>>5, mb_decoder.cpp:74-155), and mismatch
    control is a no-op for the vectors chosen (odd coefficient sums), so each block's QFS is the
    golden input exactly.  Picture 0 (I) puts the put-vectors; picture 1 (P, zero MV from
    picture 0) adds the add-vectors onto them, so the golden add output is the reference's add
    over the reference's own put output.  Hundreds of the blocks saturate int16 inside the
    transform (put_saturates), so the kernel's saturating arithmetic is what is checked."""
    import os
    from conftest import GOLDEN
    vec = np.load(os.path.join(GOLDEN, "idct_vectors.npz"))
    ch = np.load(os.path.join(GOLDEN, "idct_chain.npz"))
    F, put = vec["F"], vec["put"]
    pidx, aidx, add_exp = ch["put_idx"], ch["add_idx"], ch["add"]
    assert int(ch["put_saturates"].sum()) >= 200
    mbw, mbh = 16, 12
    w, h = mbw * 16, mbh * 16
    n = mbw * mbh
    assert len(pidx) == n * 6
    pics = np.zeros(2, R.PIC_DTYPE)
    mbs = np.zeros(2 * n, R.MB_DTYPE)
    coefs = []
    for p in range(2):
        P = pics[p]
        P["dst_slot"], P["fwd_slot"], P["bwd_slot"] = p, (0 if p else -1), -1
        P["picture_coding_type"] = 2 if p else 1
        P["mb_first"], P["mb_width"], P["mb_height"] = p * n, mbw, mbh
        P["W"] = 16
        for k in range(n):
            m = mbs[p * n + k]
            m["x"], m["y"], m["qscale"], m["cbp"] = k % mbw, k // mbw, 1, 0x3F
            m["flags"] = R._lib.MB_FWD if p else R._lib.MB_INTRA
            m["coef_off"] = len(coefs)
            for b in range(6):
                q = F[aidx[k * 6 + b]] if p else F[pidx[k * 6 + b]]
                if not p:
                    coefs.append(R._lib.coef_pack(int(q[0]), 0, b, COEF_DC, m["x"]))
                for i in range(0 if p else 1, 64):
                    v = int(q[_QFS_OF_POS[i]])
                    if v:
                        coefs.append(R._lib.coef_pack(v, i, b, 0, m["x"]))
            m["ncoef"] = len(coefs) - m["coef_off"]
    coefs = np.array(coefs, dtype=np.uint32)
    got = gpu_decode(_P(w, h, 1, pics, mbs, coefs))

    def block(planes, k, b):
        mx, my = k % mbw, k // mbw
        if b < 4:
            y0, x0 = my * 16 + (b >> 1) * 8, mx * 16 + (b & 1) * 8
            return planes[0][y0:y0 + 8, x0:x0 + 8].reshape(64)
        return planes[b - 3][my * 8:my * 8 + 8, mx * 8:mx * 8 + 8].reshape(64)

    bad_put = [j for j in range(n * 6) if not np.array_equal(block(got[0], j // 6, j % 6), put[pidx[j]])]
    bad_add = [j for j in range(n * 6) if not np.array_equal(block(got[1], j // 6, j % 6), add_exp[j])]
    assert not bad_put and not bad_add, (bad_put[:8], bad_add[:8])


@pytest.mark.gpu
def test_product_library_refuses_dev_ablations():
    """MP2VG_ABLATE (timing-only kernels with wrong output) is compiled only into dev builds
    (tools/dev_build.sh); the product library fails the decode instead of silently ablating."""
    import os
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from tiny_mp2v_dec_amd import records as R\n"
            "es = R.generate_es(width=64, height=48, chroma_format=1, n_gops=1, gop_n=3, gop_m=1, seed=7)\n"
            "p = R.Parsed(es, 64, 48, 1)\n"
            "with R.DeviceContext(64, 48, 1, slots=p.npics) as d:\n"
            "    d.upload(p.pics, p.mbs, p.coefs)\n"
            "    try:\n"
            "        d.decode(); d.synchronize()\n"
            "    except Exception as e:\n"
            "        print('refused:', e); sys.exit(0)\n"
            "sys.exit(5)\n") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MP2VG_ABLATE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "refused" in r.stdout, (r.returncode, r.stdout[-500:], r.stderr[-1500:])


def test_pool_probes_keep_the_decoded_frames():
    """The placement diagnostics (mp2vg_pool_probe: load and load+store-back sweeps per pool
    block, random and same-offset 1-KB reads over the pool, random reads inside each block) and
    the clock probe leave every decoded slot as it was, and report positive rates."""
    import ctypes
    from tiny_mp2v_dec_amd._lib import lib
    es = R.generate_es(width=176, height=144, chroma_format=1, n_gops=2, gop_n=6, gop_m=3, seed=77)
    parsed = R.Parsed(es, 176, 144, 1)
    with R.DeviceContext(176, 144, 1, slots=parsed.npics) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        before = ctx.digests(np.arange(parsed.npics))
        for mode in range(8):
            rates = ctx.pool_probe(rw=mode, reps=1)
            # (mode 5: the second record bank is allocated only once a second batch is uploaded)
            assert len(rates) >= 1 and ((rates > 0).any() if mode == 5 else (rates > 0).all()), (mode, rates)
        assert np.array_equal(ctx.digests(np.arange(parsed.npics)), before)
        exp = oracle_frames(parsed)
        for p in range(parsed.npics):
            got = ctx.download(p)
            for k in range(3):
                assert np.array_equal(got[k], exp[p][k]), (p, k)
    ghz = ctypes.c_double()
    assert lib().mp2vg_clock_probe(0, ctypes.byref(ghz)) == 0 and 0.5 < ghz.value < 4.0


def test_pool_placement_calibration_keeps_every_frame(monkeypatch):
    """The runtime's placement calibration (calibrate_placement: at a large pool's first batch the
    batch is decoded on the pool and on copies of it in fresh blocks, and the fastest pool is
    kept), forced on a small pool: batch 1 (12 I pictures) is calibrated over 3 pools, batch 2 (P
    and B pictures predicting from batch 1's slots 10 and 11) reads the kept pool; every frame of
    both vs the oracle, and the calibration ran (2 rounds x 3 candidate times)."""
    monkeypatch.setenv("MP2VG_PLACE_CANDIDATES", "3")
    monkeypatch.setenv("MP2VG_PLACE_MIN_MB", "0")
    w, h, cf = 96, 64, 1
    pics, mbs, coefs = random_batch(w, h, cf, 16, seed=8080, n_intra=12)
    exp = oracle_frames(_P(w, h, cf, pics, mbs, coefs))
    n = (w // 16) * (h // 16)
    c0 = int(mbs["coef_off"][12 * n])
    p2 = pics[12:].copy()
    p2["mb_first"] -= 12 * n
    m2 = mbs[12 * n:].copy()
    m2["coef_off"] -= c0
    with R.DeviceContext(w, h, cf, slots=16) as ctx:
        ctx.upload(pics[:12], mbs[:12 * n], coefs[:c0])
        ctx.decode()
        ctx.synchronize()
        ms, kept = ctx.placement()
        assert len(ms) == 6 and 0 <= kept < 3 and all(t > 0 for t in ms)
        ctx.upload(p2, m2, coefs[c0:])
        ctx.decode()
        ctx.synchronize()
        assert ctx.placement() == (ms, kept)  # once per context
        for p in range(16):
            got = ctx.download(p)
            for k in range(3):
                assert np.array_equal(got[k], exp[p][k]), (p, k)


@pytest.mark.parametrize("config,gops", [("c1", 120), ("c5", 64)])
def test_whole_round_i_slices_vs_reference_digests(config, gops):
    """The I-only bench batches at their bench sizes, where the planner cuts I slices across MB
    rows to fill whole rounds of resident workgroups (runtime.cpp i_slice_groups: c1 128-MB, c5
    256-MB slices): every frame's device digest == the compiled reference's
    (tests/golden/bench_digests.npz)."""
    import importlib
    bench = importlib.import_module("bench")
    width, height, cf, gparams, _ = bench.CONFIGS[config]
    es = R.generate_es(width=width, height=height, chroma_format=cf, n_gops=gops, seed=1729, **gparams)
    parsed = R.Parsed(es, width, height, cf, threads=8)
    exp = bench.expected_digests(config, gops, 1729)
    assert exp is not None
    with R.DeviceContext(width, height, cf, slots=parsed.npics) as ctx:
        ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
        ctx.decode()
        ctx.synchronize()
        dig = ctx.digests(np.arange(parsed.npics))
    assert np.array_equal(dig, exp)

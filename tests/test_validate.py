"""CPU: the record-batch validation mp2vg_batch_upload runs before any copy
(mp2vg_batch_validate, no device): batches the parser emits pass, and batches no kernel may see
are refused with MP2VG_E_INVALID."""
import numpy as np
import pytest

from tiny_mp2v_dec_amd import _lib
from tiny_mp2v_dec_amd import records as R


def _parsed(cf=1, fpfd=1, seed=5, w=176, h=144):
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=1, gop_n=12, gop_m=3,
                       frame_pred_frame_dct=fpfd, seed=seed)
    return R.Parsed(es, w, h, cf)


@pytest.mark.parametrize("cf", [1, 2, 3])
def test_parsed_batches_validate(cf):
    p = _parsed(cf, fpfd=0)
    n = R.validate_batch(p.width, p.height, cf, p.npics, p.pics, p.mbs, p.coefs)
    assert 1 <= n <= 2 * 6  # one launch per dependency level and picture set


def test_444_field_dct_record_rejected():
    """4:4:4 dct_type=1: the reference puts blocks 10/11 at (dct_type ? 1 : 8) * stride + 8 with the
    doubled luma stride (mb_decoder.cpp:193-194); the kernel's spec placement would diverge
    silently, so the upload refuses such records."""
    p = _parsed(3, fpfd=0)
    mbs = p.mbs.copy()
    coded = np.nonzero(mbs["cbp"] != 0)[0]
    assert len(coded)
    mbs["flags"][coded[0]] |= _lib.MB_DCT_FIELD
    with pytest.raises(_lib.Mp2vgError, match="4:4:4 field-DCT"):
        R.validate_batch(p.width, p.height, 3, p.npics, p.pics, mbs, p.coefs)
    # 4:2:0 / 4:2:2 field DCT is fine
    q = _parsed(2, fpfd=0)
    m2 = q.mbs.copy()
    m2["flags"][np.nonzero(m2["cbp"] != 0)[0][0]] |= _lib.MB_DCT_FIELD
    R.validate_batch(q.width, q.height, 2, q.npics, q.pics, m2, q.coefs)


def test_malformed_batches_rejected():
    p = _parsed(1)
    args = (p.width, p.height, 1, p.npics)

    def bad(pics=p.pics, mbs=p.mbs, coefs=p.coefs, nslots=p.npics, match=None):
        with pytest.raises(_lib.Mp2vgError, match=match):
            R.validate_batch(p.width, p.height, 1, nslots, pics, mbs, coefs)

    pics = p.pics.copy(); pics[1]["dst_slot"] = p.npics
    bad(pics=pics, match="slot out of range")
    mbs = p.mbs.copy(); mbs[3]["x"] += 1
    bad(mbs=mbs, match="raster order")
    mbs = p.mbs.copy(); mbs[0]["cbp"] = 1 << 6
    bad(mbs=mbs, match="cbp")
    coefs = p.coefs.copy(); coefs[0] ^= 1 << 28
    bad(coefs=coefs, match="column mod 8")
    mbs = p.mbs.copy(); k = int(np.nonzero(mbs["ncoef"])[0][-1]); mbs[k]["coef_off"] = len(p.coefs)
    bad(mbs=mbs, match="outside the batch")
    pics = p.pics.copy(); pics[1]["fwd_slot"] = -1; pics[1]["bwd_slot"] = -1
    bad(pics=pics, match="missing reference")
    # the picture type picks the launch's kernel mode and whether the picture stores anchor
    # tiles (runtime.cpp TilePlan): a type outside 1..3 would run the B kernel without storing the
    # tiles a later picture reads
    for t in (0, 4, -1):
        pics = p.pics.copy(); pics[1]["picture_coding_type"] = t
        bad(pics=pics, match="picture_coding_type")
    R.validate_batch(*args, p.pics, p.mbs, p.coefs)


def test_intra_record_contract():
    """The I kernel dequantises every word with the intra rule and, in 4:4:4, stores clamp(residual)
    with no prediction: an I picture with a non-intra MB, or an intra MB that does not code every
    block (mb_decoder.cpp codes all blocks of intra MBs), is refused."""
    p = _parsed(3)
    first_i = int(np.nonzero(p.pics["picture_coding_type"] == 1)[0][0])
    mbs = p.mbs.copy()
    k = int(p.pics[first_i]["mb_first"])
    mbs["flags"][k] = int(mbs["flags"][k]) & ~_lib.MB_INTRA
    with pytest.raises(_lib.Mp2vgError, match="non-intra macroblock in an I picture"):
        R.validate_batch(p.width, p.height, 3, p.npics, p.pics, mbs, p.coefs)
    mbs = p.mbs.copy()
    partial = np.nonzero((mbs["flags"] & _lib.MB_INTRA == 0) & (mbs["cbp"] != 0) & (mbs["cbp"] != 0xFFF))[0]
    assert len(partial)
    mbs["flags"][partial[0]] |= _lib.MB_INTRA
    with pytest.raises(_lib.Mp2vgError, match="intra macroblock whose cbp"):
        R.validate_batch(p.width, p.height, 3, p.npics, p.pics, mbs, p.coefs)


def test_coefficient_array_limit():
    """The I kernels read coefficient words through a buffer resource with 32-bit byte offsets: a
    batch of 2^30 or more words is refused before any record is read."""
    import ctypes
    p = _parsed(1)
    cfg = _lib.make_config(p.width, p.height, 1, pool=p.npics)
    vp = ctypes.c_void_p
    n = ctypes.c_int32()
    of_pic = np.zeros(len(p.pics), np.int32)
    mode = np.zeros(64, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    rc = _lib.lib().mp2vg_batch_validate(ctypes.byref(cfg), p.npics, p.pics.ctypes.data_as(vp), len(p.pics),
                                         p.mbs.ctypes.data_as(vp), len(p.mbs), p.coefs.ctypes.data_as(vp),
                                         ctypes.c_uint64(1 << 30), ctypes.byref(n), of_pic.ctypes.data_as(i32p),
                                         mode.ctypes.data_as(i32p), len(mode))
    assert rc == -1  # MP2VG_E_INVALID
    assert "coefficient words" in _lib.lib().mp2vg_last_error().decode()


@pytest.mark.parametrize("cf", [1, 2, 3])
def test_motion_vectors_outside_the_reference_rejected(cf):
    """Every vector the kernel applies must keep its reads inside the reference planes, the input
    contract the reference itself relies on (mb_decoder.cpp:212-289; the kernel's row offsets are
    not clamped into the plane): a forward or backward vector one half-pel past the left, top,
    right or bottom edge is refused, the vector at the edge is not."""
    p = _parsed(cf, fpfd=0)
    w, h = p.width, p.height
    fl = p.mbs["flags"].astype(np.int64)
    inter = np.nonzero(((fl & _lib.MB_INTRA) == 0) & ((fl & 8) == 0))[0]  # frame-MC inter MBs
    k = int(inter[0])
    s = 1 if (fl[k] & 4) and not (fl[k] & 2) else 0  # a direction this MB uses
    x, y = int(p.mbs["x"][k]), int(p.mbs["y"][k])
    R.validate_batch(w, h, cf, p.npics, p.pics, p.mbs, p.coefs)
    for mvx, mvy, ok in ((-2 * 16 * x, 0, True), (-2 * 16 * x - 1, 0, False), (0, -2 * 16 * y, True),
                         (0, -2 * 16 * y - 2, False), (2 * (w - 16 - 16 * x), 0, True),
                         (2 * (w - 16 - 16 * x) + 1, 0, False), (0, 2 * (h - 16 - 16 * y) + 2, False)):
        mbs = p.mbs.copy()
        mbs["mv"][k, 0, s] = (mvx, mvy)
        if ok:
            R.validate_batch(w, h, cf, p.npics, p.pics, mbs, p.coefs)
        else:
            with pytest.raises(_lib.Mp2vgError, match="reads outside the reference"):
                R.validate_batch(w, h, cf, p.npics, p.pics, mbs, p.coefs)


@pytest.mark.parametrize("cf,seed", [(1, 11), (2, 12), (3, 13)])
def test_parser_output_of_mutated_streams_passes_full_validation(cf, seed):
    """The drop-in uploads its own parser's records on the trusted path (only picture-level
    checks, usage and coefficient ranges: runtime.cpp uses_only), so the parser must uphold the
    whole record contract on ANY input.  Byte-mutated and truncated streams that still parse must
    produce batches that pass the full, untrusted validation (mp2vg_batch_validate)."""
    w, h = 176, 144
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=2, gop_n=6, gop_m=3,
                       frame_pred_frame_dct=0 if cf != 3 else 1, seed=seed)
    rng = np.random.default_rng(seed)
    parsed_ok = 0
    for trial in range(150):
        b = bytearray(es)
        if trial % 5 == 4:
            b = b[:int(rng.integers(len(b) // 4, len(b)))]  # truncated
        else:
            for _ in range(int(rng.integers(1, 6))):
                i = int(rng.integers(0, len(b)))
                b[i] = int(rng.integers(0, 256)) if trial % 2 else b[i] ^ (1 << int(rng.integers(0, 8)))
        try:
            p = R.Parsed(bytes(b), w, h, cf)
        except _lib.Mp2vgError:
            continue
        if p.npics == 0:
            continue
        parsed_ok += 1
        R.validate_batch(w, h, cf, p.npics, p.pics, p.mbs, p.coefs)  # raises on any violation
    assert parsed_ok > 10


def test_i_only_launch_modes():
    """Every I-only launch of a product library runs the tile-storing I kernel (mode 0); the
    tile-free I kernel (mode 4, runtime.cpp plan_batch) is a dev-build switch (MP2VG_I_TILEFREE),
    measured neutral on c1 in two rounds."""
    w, h = 176, 144
    es = R.generate_es(width=w, height=h, chroma_format=1, n_gops=16, gop_n=1, gop_m=1, seed=3)
    p = R.Parsed(es, w, h, 1)
    assert R.plan_batch(w, h, 1, p.npics, p.pics, p.mbs, p.coefs)[1].tolist() == [0, 0]
    assert R.plan_batch(w, h, 1, p.npics, p.pics, p.mbs, p.coefs, one_stream=True)[1].tolist() == [0]
    g = _parsed(1)
    modes = R.plan_batch(g.width, g.height, 1, g.npics, g.pics, g.mbs, g.coefs)[1].tolist()
    assert 0 in modes and 4 not in modes


def test_backward_prediction_in_a_p_picture_rejected():
    """The P loop predicts every non-intra MB of a P picture from the forward reference
    (recon.hip issue_pass), so a P picture whose MBs predict backward is refused."""
    p = _parsed(1)
    k = int(np.nonzero(p.pics["picture_coding_type"] == 2)[0][0])
    mbs = p.mbs.copy()
    first = int(p.pics[k]["mb_first"])
    inter = np.nonzero((mbs["flags"][first:first + 99] & _lib.MB_INTRA) == 0)[0]
    mbs["flags"][first + inter[0]] |= _lib.MB_BWD
    with pytest.raises(_lib.Mp2vgError, match="backward prediction in a P picture"):
        R.validate_batch(p.width, p.height, 1, p.npics, p.pics, mbs, p.coefs)

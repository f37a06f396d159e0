"""CPU: the host emitter's stream headers (mp2vg_parsed_stream_headers, the drop-in's
m_sequence_header & co.) equal the REAL reference decoder's public header members
(decoder.h:124-130) after decode(), on every golden stream and on a header-syntax variant
(matrices in the sequence header, two sequence_display_extensions, user data, a second GOP
header) -- fixtures from tests/golden/make_header_fixtures.py; and the shard split used for GOP
sharding (mp2vg_parsed_shards) follows the streams' reference structure."""
import json
import os

import numpy as np
import pytest

from tiny_mp2v_dec_amd import records as R

HERE = os.path.dirname(os.path.abspath(__file__))
STREAMS = os.path.join(HERE, "golden", "streams")
FIX = json.load(open(os.path.join(HERE, "golden", "stream_headers.json")))
MANIFEST = {m["name"]: m for m in json.load(open(os.path.join(STREAMS, "manifest.json")))}


def _geometry(name):
    if name in MANIFEST:
        m = MANIFEST[name]
        return m["file"], m["width"], m["height"], m["chroma_format"]
    d = FIX[name]
    return d["file"], d["width"], d["height"], d["chroma_format"]


def _as_dict(st):
    out = {}
    for f, _ in st._fields_:
        v = getattr(st, f)
        out[f] = list(v) if hasattr(v, "__len__") else int(v)
    return out


@pytest.mark.parametrize("name", sorted(FIX))
def test_stream_headers_match_reference(name):
    f, w, h, cf = _geometry(name)
    es = open(os.path.join(STREAMS, f), "rb").read()
    p = R.Parsed(es, w, h, cf)
    exp = FIX[name]
    hd = p.headers
    sh = _as_dict(hd.sequence_header)
    for k, v in exp["sequence_header"].items():
        assert sh[k] == v, (k, sh[k], v)
    assert _as_dict(hd.sequence_extension) == exp["sequence_extension"]
    if exp["sequence_display_extension"] is None:
        assert hd.have_sequence_display_extension == 0
    else:
        assert hd.have_sequence_display_extension == 1
        assert _as_dict(hd.sequence_display_extension) == exp["sequence_display_extension"]
    if exp["group_of_pictures_header"] is None:
        assert hd.have_group_of_pictures_header == 0
    else:
        assert hd.have_group_of_pictures_header == 1
        assert _as_dict(hd.group_of_pictures_header) == exp["group_of_pictures_header"]
    assert exp["sequence_scalable_extension"] is None and exp["user_data_len"] == 0
    assert p.npics == exp["frames"]


def test_shards_closed_gops_are_gops():
    """Closed GOPs (leading B pictures predict only from their own I) are independent shards."""
    m = MANIFEST["ipb420_qcif"]
    p = R.Parsed(open(os.path.join(STREAMS, m["file"]), "rb").read(), m["width"], m["height"], 1)
    assert p.nshards == 2
    assert np.array_equal(p.shard, p.gop)


def test_shards_respect_every_reference():
    """No macroblock predicts from a picture of another shard, and shards are decode-order runs.
    The one picture-level reference that may cross is a closed GOP's leading B picture's
    forward anchor, which none of its macroblocks reads."""
    crossed = 0
    for name in ("ipb420_qcif", "ipb420_qcif_openb", "stress_mv_fcode4", "tall_2816_vpos_ext", "hdr_variant"):
        f, w, h, cf = _geometry(name)
        p = R.Parsed(open(os.path.join(STREAMS, f), "rb").read(), w, h, cf)
        assert np.all(np.diff(p.shard) >= 0) and p.shard[0] == 0 and p.nshards == p.shard[-1] + 1
        n = int(p.pics[0]["mb_width"]) * int(p.pics[0]["mb_height"])
        for i, pic in enumerate(p.pics):
            fwd, bwd = int(pic["fwd_slot"]), int(pic["bwd_slot"])
            assert bwd < 0 or p.shard[bwd] == p.shard[i]
            if fwd >= 0 and p.shard[fwd] != p.shard[i]:
                crossed += 1
                assert int(pic["picture_coding_type"]) == 3 and p.shard[bwd] == p.shard[i]
                fl = p.mbs["flags"][i * n:(i + 1) * n].astype(np.int64)
                uses_fwd = ((fl & 1) == 0) & (((fl & 2) != 0) | ((fl & 4) == 0))
                assert not uses_fwd.any()
    assert crossed > 0  # ipb420_qcif's second GOP opens with backward-only B pictures


def test_shards_of_a_long_closed_gop_stream():
    es = R.generate_es(width=176, height=144, chroma_format=1, n_gops=7, gop_n=12, gop_m=3, leading_b=1, seed=5)
    p = R.Parsed(es, 176, 144, 1)
    assert p.nshards == 7 and np.array_equal(p.shard, p.gop)

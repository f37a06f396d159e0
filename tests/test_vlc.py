"""CPU: every Annex B VLC entry pinned to the REAL reference decoders.

tests/golden/vlc_vectors.npz holds, for every code of the reference's tables followed by 32
random suffixes, what the reference's decoders (mp2v_vlc_dec.hpp:36-267) return and how many bits
they consume (tests/golden/make_vlc_vectors.py, after test/gtest/cavlc/cavlc_test.cpp:25-88).
The host emitter's own LUTs (built from vlc_tables.h) decode the same bits through
mp2vg_vlc_decode and must agree entry by entry -- value and consumed length -- so a wrong
vlc_tables.h entry fails here even if the stream writer never emits it.

Where the emitter reads more than the reference's table decoder, the difference is the next
syntax element and is checked as such: the motion_code sign bit is part of the reference's B.10
codes too (value signed, same length); DCT coefficients: the emitter also consumes the sign bit
that follows (the reference's parse_block reads it, mb_decoder.cpp:74-155), so its length is one
more and its level carries the sign of the suffix's first bit.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN
from tiny_mp2v_dec_amd import _lib

V = np.load(os.path.join(GOLDEN, "vlc_vectors.npz"))
TABLES = {0: "MBA B.1 (lut)", 10: "MBA B.1", 1: "macroblock_type I B.2", 2: "macroblock_type P B.3",
          3: "macroblock_type B B.4", 4: "coded_block_pattern B.9", 5: "motion_code B.10",
          6: "dct_dc_size_luminance B.12", 7: "dct_dc_size_chrominance B.13", 8: "DCT coefficients B.14",
          9: "DCT coefficients B.15"}


def ours(table, bits):
    v, a, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    rc = _lib.lib().mp2vg_vlc_decode(table, int(bits), ctypes.byref(v), ctypes.byref(a), ctypes.byref(n))
    return rc, v.value, a.value, n.value


def test_vectors_cover_every_reference_table_entry():
    sizes = {0: 33, 10: 33, 1: 2, 2: 7, 3: 11, 4: 64, 5: 33, 6: 12, 7: 12, 8: 111, 9: 111, 11: 3}
    for t, n in sizes.items():
        sel = V["table"] == t
        assert len(set(V["entry"][sel].tolist())) == n, t
    assert np.all(V["consumed"] == V["code_len"])  # the reference consumes exactly the code


@pytest.mark.parametrize("table", sorted(TABLES), ids=[TABLES[t] for t in sorted(TABLES)])
def test_host_vlc_decoders_match_reference(table):
    sel = np.nonzero(V["table"] == table)[0]
    our_table = 0 if table == 10 else table
    bad = []
    for i in sel:
        bits, val, aux, n = int(V["bits"][i]), int(V["value"][i]), int(V["aux"][i]), int(V["consumed"][i])
        rc, v, a, m = ours(our_table, bits)
        if table in (8, 9):  # + the sign bit: level sign = the bit after the code
            sign = (bits >> (63 - n)) & 1
            exp = (0, val, -aux if sign else aux, n + 1)
        else:
            exp = (0, val, 0, n)
        if (rc, v, a, m) != exp:
            bad.append((int(V["entry"][i]), hex(bits), exp, (rc, v, a, m)))
    assert not bad, bad[:5]


def test_escape_eob_and_invalid_codes():
    """Codes outside the reference's tables, with the emitter's semantics: macroblock_escape (B.1),
    end_of_block (B.14 '10', B.15 '0110'), the coefficient escape '000001' + 6-bit run + signed
    12-bit level (ISO 13818-2 7.2.2.3; reference mb_decoder.cpp:74-155), and invalid codes."""
    def window(s):
        return int(s.ljust(64, "0"), 2)
    assert ours(0, window("00000001000" + "1"))[1:] == (-33, 0, 11)
    assert ours(8, window("10"))[1:] == (-1, 0, 2)
    assert ours(9, window("0110"))[1:] == (-1, 0, 4)
    for tab in (8, 9):
        for run, level in ((0, 1), (5, -7), (63, 2047), (31, -2047), (0, -2048 + 1)):
            code = "000001" + format(run, "06b") + format(level & 0xFFF, "012b")
            assert ours(tab, window(code + "1"))[1:] == (run, level, 24), (tab, run, level)
    assert ours(4, window("000000000" + "0"))[0] == -6  # cbp '0000 0000 0' is forbidden
    assert ours(5, window("0000000000" + "0"))[0] == -6

"""Per-entry Annex B VLC vectors from the REAL reference decoders.

Run in the build container (needs oracle/_ref/ref_vlc, built from /root/reference by
`make -C oracle ref`).  ref_vlc feeds every code of the reference's own tables (mp2v_luts.hpp:
B.1 MBA, B.2-B.4 macroblock_type, B.9 cbp, B.10 motion_code, B.11 dmvector, B.12/B.13
dct_dc_size, B.14/B.15 DCT coefficients) followed by 32 random suffixes through the reference's
decoders (mp2v_vlc_dec.hpp:36-267) and records the decoded value and consumed length, as the
reference's conformance test does (test/gtest/cavlc/cavlc_test.cpp:25-88).  Saved as
tests/golden/vlc_vectors.npz; tests/test_vlc.py decodes the same bits with the host emitter's
LUTs (mp2vg_vlc_decode).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "ref_vlc")
REC = np.dtype([("table", "<i4"), ("entry", "<i4"), ("bits", "<u8"), ("value", "<i4"), ("aux", "<i4"),
                ("consumed", "<i4"), ("code_len", "<i4")])


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "vlc.bin")
        subprocess.check_call([REF, out, "32", "1729"])
        r = np.fromfile(out, REC)
    np.savez_compressed(os.path.join(HERE, "vlc_vectors.npz"), **{k: r[k] for k in REC.names})
    print(len(r), "vectors")


if __name__ == "__main__":
    main()

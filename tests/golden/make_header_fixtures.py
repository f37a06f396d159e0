"""Generate the stream-header golden fixtures from the REAL reference decoder.

Run in the build container (needs oracle/_ref/ref_decode, built from /root/reference by
`make -C oracle ref`).  The reference keeps the sequence-level headers as public members of
mp2v_decoder_c (decoder.h:124-130, parsed by mp2v_hdr.cpp:4-83); ref_decode's ".hdr.json" mode
dumps them after decode().  Cases:
  * every golden stream of tests/golden/streams/manifest.json;
  * hdr_variant.m2v: ipb420_qcif with its sequence header replaced by one that loads both
    matrices (other field values too), and a sequence_display_extension (colour description on),
    a second one (colour description off: the later one wins), a user_data block and a second
    GOP header with another time code spliced in -- header syntax the stream writer never emits.
Writes tests/golden/stream_headers.json {name: headers} and tests/golden/streams/hdr_variant.m2v.
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref", "ref_decode")
STREAMS = os.path.join(HERE, "streams")


class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, value, n):
        self.v = (self.v << n) | (value & ((1 << n) - 1))
        self.n += n

    def bytes(self):
        pad = (-self.n) % 8
        return (self.v << pad).to_bytes((self.n + pad) // 8, "big")


def start_codes(es):
    out, k = [], 0
    while True:
        k = es.find(b"\x00\x00\x01", k)
        if k < 0:
            return out
        out.append(k)
        k += 3


def sequence_header(w, h, rng):
    b = Bits()
    b.put(0x1B3, 32)
    b.put(w, 12)
    b.put(h, 12)
    b.put(2, 4)  # aspect_ratio_information
    b.put(5, 4)  # frame_rate_code
    b.put(0x12345, 18)
    b.put(1, 1)  # marker
    b.put(0x155, 10)
    b.put(1, 1)  # constrained_parameters_flag
    for _ in range(2):  # load_intra / load_non_intra quantiser matrix, each with 64 bytes
        b.put(1, 1)
        for v in rng.integers(1, 256, 64):
            b.put(int(v), 8)
    return b.bytes()


def display_extension(colour, hsize, vsize):
    b = Bits()
    b.put(0x1B5, 32)
    b.put(2, 4)
    b.put(5, 3)  # video_format
    b.put(1 if colour else 0, 1)
    if colour:
        b.put(1, 8)
        b.put(6, 8)
        b.put(4, 8)
    b.put(hsize, 14)
    b.put(1, 1)
    b.put(vsize, 14)
    return b.bytes()


def gop_header(time_code, closed, broken):
    b = Bits()
    b.put(0x1B8, 32)
    b.put(time_code, 25)
    b.put(closed, 1)
    b.put(broken, 1)
    return b.bytes()


def variant(es, w, h):
    rng = np.random.default_rng(1750)
    sc = start_codes(es)
    codes = [es[k + 3] for k in sc]
    i_seq = codes.index(0xB3)
    i_ext = codes.index(0xB5, i_seq)  # the sequence_extension right after it
    i_gop2 = [i for i, c in enumerate(codes) if c == 0xB8][1]
    seq_end = sc[i_ext]
    ext_end = sc[i_ext + 1]
    out = (es[:sc[i_seq]] + sequence_header(w, h, rng) + es[seq_end:ext_end] +
           display_extension(True, w - 16, h - 16) + b"\x00\x00\x01\xb2user data bytes" +
           display_extension(False, w, h) + es[ext_end:sc[i_gop2]] +
           gop_header(0x0ABCDE, 1, 0) + es[sc[i_gop2 + 1]:])
    return out


def ref_headers(path, w, h, cf):
    out = path + ".hdr.json"
    r = subprocess.run([REF, path, str(w), str(h), str(cf), "1", out], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference failed on {path}: {r.stderr[-300:]}")
    with open(out) as fh:
        d = json.load(fh)
    os.unlink(out)
    d["sequence_header"].pop("_", None)
    d["frames"] = json.loads(r.stdout.strip().splitlines()[-1])["frames"]
    return d


def main():
    if not os.path.exists(REF):
        sys.exit("oracle/_ref/ref_decode missing: make -C oracle ref")
    manifest = json.load(open(os.path.join(STREAMS, "manifest.json")))
    res = {}
    for m in manifest:
        res[m["name"]] = ref_headers(os.path.join(STREAMS, m["file"]), m["width"], m["height"], m["chroma_format"])
    base = next(m for m in manifest if m["name"] == "ipb420_qcif")
    es = open(os.path.join(STREAMS, base["file"]), "rb").read()
    path = os.path.join(STREAMS, "hdr_variant.m2v")
    with open(path, "wb") as fh:
        fh.write(variant(es, base["width"], base["height"]))
    d = ref_headers(path, base["width"], base["height"], base["chroma_format"])
    d["file"], d["width"], d["height"], d["chroma_format"] = "hdr_variant.m2v", base["width"], base["height"], 1
    res["hdr_variant"] = d
    with open(os.path.join(HERE, "stream_headers.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(f"{len(res)} header fixtures; variant frames {d['frames']}")


if __name__ == "__main__":
    main()

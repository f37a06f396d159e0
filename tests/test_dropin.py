"""GPU: the drop-in decoder API (reference mp2v_decoder_c / frame_c / decoder_config_t) decodes the
golden streams to the reference's exact YUV, in the reference's display order, on a render thread."""
import hashlib
import os
import subprocess
import threading

import pytest

from conftest import STREAMS, load_manifest, read_stream
from tiny_mp2v_dec_amd import build as B
from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c

pytestmark = pytest.mark.gpu
MANIFEST = load_manifest()


@pytest.mark.parametrize("entry", [e for e in MANIFEST if e["width"] <= 352], ids=lambda e: e["name"])
def test_dropin_python_api(entry):
    md5, types, threads = [], [], set()

    def render(frame):
        threads.add(threading.get_ident())
        assert frame.get_strides(0) % 64 == 0 and frame.get_strides(1) % 64 == 0
        md5.append(hashlib.md5(frame.yuv_bytes()).hexdigest())
        types.append(frame.picture_coding_type)

    cfg = decoder_config_t(entry["width"], entry["height"], entry["chroma_format"], pictures_pool_size=10,
                           num_threads=4)
    dec = mp2v_decoder_c(cfg, render)
    es = read_stream(entry)
    assert dec.decode(es, len(es))
    dec.close()
    assert md5 == entry["md5"]
    assert threading.get_ident() not in threads  # callbacks ran on the render thread


def test_dropin_cpp_cli_matches_reference(tmp_path):
    e = next(m for m in MANIFEST if m["name"] == "hd1080_420_ipb")
    out = tmp_path / "o.yuv"
    r = subprocess.run([B.CLI, "-v", os.path.join(STREAMS, e["file"]), "-o", str(out), "-w", "1920", "-h", "1088",
                        "-c", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Time =" in r.stdout
    data = out.read_bytes()
    fb = 1920 * 1088 * 3 // 2
    assert [hashlib.md5(data[k * fb:(k + 1) * fb]).hexdigest() for k in range(len(data) // fb)] == e["md5"]


def test_dropin_long_stream_recycles_slots():
    """More pictures than the chunk/pool: slots are recycled once no later picture predicts."""
    from helpers import oracle_frames, yuv_md5
    from tiny_mp2v_dec_amd.records import Parsed, generate_es
    es = generate_es(width=176, height=144, chroma_format=2, n_gops=4, gop_n=12, gop_m=3, seed=31)
    parsed = Parsed(es, 176, 144, 2)
    exp = [yuv_md5(oracle_frames(parsed)[d]) for d in parsed.display]
    got = []
    dec = mp2v_decoder_c(decoder_config_t(176, 144, 2, pictures_pool_size=4),
                         lambda f: got.append(hashlib.md5(f.yuv_bytes()).hexdigest()))
    dec.decode(es)
    dec.close()
    assert got == exp


def test_dropin_decoder_reused_across_streams():
    """One decoder, consecutive decode() calls: the persistent pinned frame pool, the two pinned
    record sets and the two device record banks carry over between calls (decoder.cpp,
    runtime.cpp), and every call still renders the oracle's frames in display order."""
    from helpers import oracle_frames, yuv_md5
    from tiny_mp2v_dec_amd.records import Parsed, generate_es
    streams = [generate_es(width=176, height=144, chroma_format=1, n_gops=n, gop_n=12, gop_m=3, seed=s)
               for n, s in ((5, 41), (2, 42), (7, 43))]
    got = []
    dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, pictures_pool_size=4, num_threads=3),
                         lambda f: got.append(hashlib.md5(f.yuv_bytes()).hexdigest()))
    for es in streams:
        parsed = Parsed(es, 176, 144, 1)
        exp = [yuv_md5(oracle_frames(parsed)[d]) for d in parsed.display]
        got.clear()
        dec.decode(es)
        assert got == exp
    dec.close()


def test_dropin_bad_stream_fails_cleanly_then_recovers():
    """A stream that breaks early (picture 2) and one that breaks at its end: decode() reports the
    error (while parse workers are still ahead of the chunk loop, parse.cpp's window and stop
    flag), and the same decoder then decodes a good stream to the oracle's frames."""
    from helpers import oracle_frames, yuv_md5
    from tiny_mp2v_dec_amd.records import Parsed, generate_es
    good = generate_es(width=176, height=144, chroma_format=1, n_gops=8, gop_n=12, gop_m=3, seed=51)
    starts = [i for i in range(len(good) - 4) if good[i:i + 4] == b"\x00\x00\x01\x01"]
    assert len(starts) > 3
    early = bytearray(good)
    early[starts[2] + 8:starts[2] + 40] = bytes(32)  # picture 2, first slice: zeros -> bad MBA code
    late = good[:starts[-1] + 12]                     # last slice cut short
    got = []
    dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, pictures_pool_size=4, num_threads=4),
                         lambda f: got.append(hashlib.md5(f.yuv_bytes()).hexdigest()))
    for bad in (bytes(early), late):
        with pytest.raises(Exception):
            dec.decode(bad)
    parsed = Parsed(good, 176, 144, 1)
    exp = [yuv_md5(oracle_frames(parsed)[d]) for d in parsed.display]
    got.clear()
    dec.decode(good)
    dec.close()
    assert got == exp


def test_dropin_device_frames_match_host_frames():
    """MP2VG_DECODER_DEVICE_FRAMES (the opt-in device-pointer output path, SURVEY §8b Output):
    frames handed over in HBM, in the same display order and byte for byte the same as the host
    frames of the reference's frame_c contract (which test_dropin_python_api pins to the
    reference)."""
    import hashlib
    from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c
    e = next(m for m in MANIFEST if m["name"] == "ipb420_qcif")
    es = read_stream(e)
    out = {}
    for dev in (False, True):
        got = []

        def render(frame, got=got, dev=dev):
            assert frame.is_device == dev
            if dev:
                assert frame.device_ptr(0)
            got.append((frame.decode_index, hashlib.md5(frame.yuv_bytes()).hexdigest()))

        d = mp2v_decoder_c(decoder_config_t(e["width"], e["height"], e["chroma_format"], device_frames=dev), render)
        d.decode(es, len(es))
        d.close()
        out[dev] = got
    assert len(out[True]) == e["frames"]
    assert out[True] == out[False]

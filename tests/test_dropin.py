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


@pytest.mark.parametrize("dl_kernel", ["1", "0"], ids=["copy_kernel", "dma"])
def test_dropin_cpp_cli_matches_reference(tmp_path, dl_kernel):
    """Frames come back by the copy kernel (default) or, with MP2VG_DL_KERNEL=0, one DMA per frame."""
    e = next(m for m in MANIFEST if m["name"] == "hd1080_420_ipb")
    out = tmp_path / "o.yuv"
    r = subprocess.run([B.CLI, "-v", os.path.join(STREAMS, e["file"]), "-o", str(out), "-w", "1920", "-h", "1088",
                        "-c", "1"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MP2VG_DL_KERNEL=dl_kernel))
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


def _oracle_md5(es, w, h, cf):
    from helpers import oracle_frames, yuv_md5
    from tiny_mp2v_dec_amd.records import Parsed
    parsed = Parsed(es, w, h, cf)
    return [yuv_md5(oracle_frames(parsed)[d]) for d in parsed.display], parsed


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_dropin_gop_sharding_over_device_lanes(devices):
    """GOP sharding (mp2vg_decoder_create_multi): the stream's independent shards are dealt to
    device lanes round-robin -- here several lanes on the one GPU, each with its own context,
    slots, banks and streams -- and the renderer still gets the oracle's frames in the
    reference's display order, with every lane used.  Closed GOPs with backward-only leading B
    pictures shard per GOP although those pictures name the previous GOP's anchor."""
    from tiny_mp2v_dec_amd.records import generate_es
    es = generate_es(width=176, height=144, chroma_format=1, n_gops=7, gop_n=12, gop_m=3, leading_b=1, seed=61)
    exp, parsed = _oracle_md5(es, 176, 144, 1)
    assert parsed.nshards == 7
    got, order = [], []
    dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, pictures_pool_size=4, num_threads=4, devices=devices),
                         lambda f: (got.append(hashlib.md5(f.yuv_bytes()).hexdigest()), order.append(f.decode_index)))
    dec.decode(es)
    lanes = dec.lane_frames()
    dec.close()
    assert got == exp and order == list(parsed.display)
    # shards merge into runs of >= 16 pictures (two 12-picture GOPs each, the last GOP alone) and
    # run r goes to lane r % n
    n = len(devices)
    runs = [24, 24, 24, 12]
    assert lanes == [sum(runs[r] for r in range(i, len(runs), n)) for i in range(n)]


def test_dropin_lane_handoff_does_not_wait_for_the_lane_left():
    """A lane change no longer blocks the host on the lane just left (decoder.cpp: its last chunk
    stays in flight until its downloads have landed, checked without waiting; the host waits on
    another lane only when the frame pool could not give the next chunk its frames).  1080p
    frames over three lanes on the one GPU: every lane change is either left in flight or
    completed without a wait, frames are the oracle's in display order (digests), and the pool
    keeps its reserved size."""
    from tiny_mp2v_dec_amd.records import generate_es
    import numpy as np
    from tiny_mp2v_dec_amd import records as R
    es = generate_es(width=1920, height=1088, chroma_format=1, n_gops=6, gop_n=12, gop_m=3, seed=71)
    parsed = R.Parsed(es, 1920, 1088, 1)
    from helpers import oracle_frames
    exp_frames = oracle_frames(parsed)
    exp = [R.planes_digest(exp_frames[d]) for d in parsed.display]
    got = []

    def render(f):
        got.append(R.planes_digest([np.array(f.get_planes(i)[:, :f.get_width(i)]) for i in range(3)]))

    dec = mp2v_decoder_c(decoder_config_t(1920, 1088, 1, num_threads=6, devices=[0, 0, 0]), render)
    before = dec.frames_allocated()
    dec.decode(es)
    in_flight, blocks, landed, changes = dec.handoff_stats()
    after = dec.frames_allocated()
    lanes = dec.lane_frames()
    dec.close()
    assert got == exp
    assert after == before
    assert lanes == [24, 24, 24]  # three runs of two 12-picture GOPs
    # two lane changes, each left in flight, found landed by the non-blocking check, or waited
    # for (a block): a host wait outside those paths would leave a change unaccounted
    assert changes == 2
    assert in_flight + landed <= changes <= in_flight + landed + blocks
    if blocks == 0:
        assert in_flight + landed == changes


def test_dropin_lanes_long_gops_bounded_pool_and_i_only():
    """Two lanes on long closed GOPs (96 pictures, longer than the 72-frame pool) keep the frame pool
    at its reserved size -- a lane's last chunk completes when the stream moves to the other lane,
    so display order never waits on an idle lane -- and an I-only stream (one shard per picture)
    is dealt in whole runs, both lanes used, frames in display order and oracle-exact."""
    from tiny_mp2v_dec_amd.records import generate_es
    for kw, nshards in ((dict(n_gops=3, gop_n=96, gop_m=3), 3), (dict(n_gops=40, gop_n=1, gop_m=1, mix=1), 40)):
        es = generate_es(width=176, height=144, chroma_format=1, seed=65, **kw)
        exp, parsed = _oracle_md5(es, 176, 144, 1)
        assert parsed.nshards == nshards
        got = []
        dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, num_threads=4, devices=[0, 0]),
                             lambda f: got.append(hashlib.md5(f.yuv_bytes()).hexdigest()))
        before = dec.frames_allocated()
        dec.decode(es)
        after = dec.frames_allocated()
        lanes = dec.lane_frames()
        dec.close()
        assert got == exp
        assert after == before, (kw, before, after)
        assert all(n > 0 for n in lanes) and sum(lanes) == parsed.npics
        if nshards == 40:  # runs of 16, 16, 8 pictures
            assert lanes == [24, 16]


def test_dropin_gop_sharding_golden_and_open_gop():
    """Golden streams through two lanes give the reference's MD5s: the closed-GOP stream is two
    12-picture shards, which merge into one run (runs are at least a 16-picture chunk), and the
    open-GOP stream is one shard (its B pictures predict across the GOP); both stay on lane 0
    (streams that do split over lanes: test_dropin_gop_sharding_over_device_lanes)."""
    from tiny_mp2v_dec_amd.records import Parsed
    for name, nshards in (("ipb420_qcif", 2), ("ipb420_qcif_openb", 1)):
        e = next(m for m in MANIFEST if m["name"] == name)
        es = read_stream(e)
        got = []
        dec = mp2v_decoder_c(decoder_config_t(e["width"], e["height"], e["chroma_format"], devices=[0, 0]),
                             lambda f: got.append(hashlib.md5(f.yuv_bytes()).hexdigest()))
        dec.decode(es, len(es))
        lanes = dec.lane_frames()
        dec.close()
        assert got == e["md5"], name
        assert Parsed(es, e["width"], e["height"], e["chroma_format"]).nshards == nshards
        assert lanes == [len(e["md5"]), 0], (name, lanes)


def test_dropin_gop_sharding_device_frames():
    """Device frames (MP2VG_DECODER_DEVICE_FRAMES) from two lanes: each frame lives on its lane's
    device pool, and the bytes and order equal the single-lane host frames."""
    from tiny_mp2v_dec_amd.records import generate_es
    es = generate_es(width=176, height=144, chroma_format=2, n_gops=4, gop_n=12, gop_m=3, leading_b=1, seed=62)
    out = {}
    for devs, dev_frames in (([0], False), ([0, 0], True)):
        got = []
        dec = mp2v_decoder_c(decoder_config_t(176, 144, 2, devices=devs, device_frames=dev_frames),
                             lambda f, got=got: got.append((f.decode_index, hashlib.md5(f.yuv_bytes()).hexdigest())))
        dec.decode(es)
        dec.close()
        out[dev_frames] = got
    assert out[True] == out[False] and len(out[True]) == 48


def test_dropin_slow_renderer_bounds_the_frame_pool():
    """A renderer slower than the GPU back-pressures the decoder (the reference blocks on its fixed
    picture pool, threads.cpp:164-166): the frame pool stays at its reserved size however long
    the stream, and the frames are still right."""
    import time
    from tiny_mp2v_dec_amd.records import generate_es
    es = generate_es(width=176, height=144, chroma_format=1, n_gops=10, gop_n=12, gop_m=3, seed=63)
    exp, _ = _oracle_md5(es, 176, 144, 1)
    got = []

    def render(f):
        time.sleep(0.004)
        got.append(hashlib.md5(f.yuv_bytes()).hexdigest())

    dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, num_threads=4), render)
    before = dec.frames_allocated()
    dec.decode(es)
    after = dec.frames_allocated()
    dec.close()
    assert got == exp
    assert before == after == 2 * 16 + 4


def test_dropin_errors_return_frames_to_the_pool():
    """Frames an error leaves in flight go back to the pool: repeated failing decodes do not grow
    a long-lived decoder."""
    from tiny_mp2v_dec_amd.records import generate_es
    good = generate_es(width=176, height=144, chroma_format=1, n_gops=8, gop_n=12, gop_m=3, seed=64)
    late = good[:[i for i in range(len(good) - 4) if good[i:i + 4] == b"\x00\x00\x01\x01"][-1] + 12]
    dec = mp2v_decoder_c(decoder_config_t(176, 144, 1, num_threads=4), lambda f: None)
    n0 = dec.frames_allocated()
    for _ in range(3):
        with pytest.raises(Exception):
            dec.decode(late)
    assert dec.frames_allocated() == n0
    dec.close()


@pytest.mark.parametrize("name", ["hdr_variant", "ipb420_qcif", "stress_mv_fcode4"])
def test_dropin_cpp_header_members_match_reference(tmp_path, name):
    """The C++ drop-in's public header members (m_sequence_header, m_sequence_extension,
    m_sequence_display_extension, m_group_of_pictures_header, user_data; reference
    decoder.h:124-130) after decode() equal the compiled reference's own members on the same
    stream (tests/golden/stream_headers.json); decoded over two device lanes."""
    import json
    fix = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "stream_headers.json")))[name]
    e = next((m for m in MANIFEST if m["name"] == name), None) or fix
    hdr = tmp_path / "h.json"
    r = subprocess.run([B.CLI, "-v", os.path.join(STREAMS, e["file"]), "-o", str(tmp_path / "o.yuv"), "-w",
                        str(e["width"]), "-h", str(e["height"]), "-c", str(e["chroma_format"]), "-d", "0,0", "-H",
                        str(hdr)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(hdr.read_text())
    exp = {k: v for k, v in fix.items() if k not in ("frames", "file", "width", "height", "chroma_format")}
    assert got == exp

"""Host side of the record path: stream generation, ES -> records parsing, and the device
context (frame pool + record batch + level-scheduled launches), mirroring the reference's
mp2v_decoder_c / frame_c vocabulary where it has one.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import MB_DTYPE, PIC_DTYPE, check, lib


def gen_params(**kw):
    p = _lib.GenParams()
    lib().mp2vg_gen_default_params(ctypes.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, v)
    return p


def _copy_out(ptr, nbytes, dtype=np.uint8):
    """Copy nbytes at a library-owned pointer into a new array.  ctypes.string_at takes a C int size,
    which goes negative (or wraps) past 2 GiB; a numpy view over the pointer has no such limit."""
    if not nbytes:
        return np.zeros(0, dtype)
    raw = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))
    return raw.view(dtype).copy()


def generate_es(**kw):
    """Write a synthetic elementary stream of the reference's decodable subset (bytes)."""
    p = gen_params(**kw)
    ptr, n = ctypes.c_void_p(), ctypes.c_uint64()
    check(lib().mp2vg_generate_es(ctypes.byref(p), ctypes.byref(ptr), ctypes.byref(n)), "generate_es")
    try:
        return _copy_out(ptr, n.value).tobytes()
    finally:
        lib().mp2vg_free(ptr)


def check_count(status, what):
    """An entry point that returns a count (>= 0) or an MP2VG_E_* status."""
    if status < 0:
        check(status, what)
    return status


class Parsed:
    """Records of a whole elementary stream (pictures in decode order; slot = decode index)."""

    def __init__(self, es: bytes, width, height, chroma_format, threads=0, reordering=True):
        self.width, self.height, self.chroma_format = width, height, chroma_format
        cfg = _lib.make_config(width, height, chroma_format, threads=threads, reordering=reordering)
        buf = np.frombuffer(es, dtype=np.uint8)
        h = ctypes.c_void_p()
        check(lib().mp2vg_parse_es(buf.ctypes.data_as(ctypes.c_void_p), len(es), ctypes.byref(cfg),
                                   ctypes.byref(h)), "parse_es")
        try:
            npics, nmbs, ncoefs = ctypes.c_int32(), ctypes.c_uint64(), ctypes.c_uint64()
            lib().mp2vg_parsed_counts(h, ctypes.byref(npics), ctypes.byref(nmbs), ctypes.byref(ncoefs))
            n, m, c = npics.value, nmbs.value, ncoefs.value
            self.pics = _copy_out(lib().mp2vg_parsed_pictures(h), n * 288, PIC_DTYPE)
            self.mbs = _copy_out(lib().mp2vg_parsed_mbs(h), m * 32, MB_DTYPE)
            self.coefs = _copy_out(lib().mp2vg_parsed_coefs(h), c * 4, np.uint32)
            order = (ctypes.c_int32 * max(n, 1))()
            lib().mp2vg_parsed_display_order(h, order, n)
            self.display = np.array(order[:n], dtype=np.int32)
            gop = (ctypes.c_int32 * max(n, 1))()
            lib().mp2vg_parsed_gop_index(h, gop, n)
            self.gop = np.array(gop[:n], dtype=np.int32)
            shard = (ctypes.c_int32 * max(n, 1))()
            self.nshards = check_count(lib().mp2vg_parsed_shards(h, shard, n), "parsed_shards")
            self.shard = np.array(shard[:n], dtype=np.int32)
            self.headers = _lib.StreamHeaders()
            check(lib().mp2vg_parsed_stream_headers(h, ctypes.byref(self.headers)), "parsed_stream_headers")
        finally:
            lib().mp2vg_parsed_free(h)

    @property
    def npics(self):
        return len(self.pics)


def plan_batch(width, height, chroma_format, nslots, pics, mbs, coefs, one_stream=False):
    """mp2vg_batch_validate: the upload's host-side record validation and launch planning, with no
    device.  Returns (launch index of each picture, kernel mode of each launch: 0 I, 1 P, 2 B,
    3 mixed, 4 I without tile stores); raises Mp2vgError for a batch the upload would refuse."""
    cfg = _lib.make_config(width, height, chroma_format, pool=nslots,
                           flags=_lib.MP2VG_CTX_ONE_STREAM if one_stream else 0)
    pics = np.ascontiguousarray(pics, PIC_DTYPE)
    mbs = np.ascontiguousarray(mbs, MB_DTYPE)
    coefs = np.ascontiguousarray(coefs, np.uint32)
    vp = ctypes.c_void_p
    n = ctypes.c_int32()
    of_pic = np.zeros(len(pics), np.int32)
    mode = np.zeros(4096, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    check(lib().mp2vg_batch_validate(ctypes.byref(cfg), nslots, pics.ctypes.data_as(vp), len(pics),
                                     mbs.ctypes.data_as(vp), len(mbs),
                                     coefs.ctypes.data_as(vp) if len(coefs) else None, len(coefs),
                                     ctypes.byref(n), of_pic.ctypes.data_as(i32p), mode.ctypes.data_as(i32p),
                                     len(mode)), "batch_validate")
    return of_pic, mode[:min(n.value, len(mode))].copy()


def validate_batch(width, height, chroma_format, nslots, pics, mbs, coefs):
    """Number of kernel launches of a valid batch (plan_batch); raises Mp2vgError otherwise."""
    return len(plan_batch(width, height, chroma_format, nslots, pics, mbs, coefs)[1])


class DeviceContext:
    """mp2vg_ctx_t: a frame pool in HBM plus a resident record batch on one GPU."""

    def __init__(self, width, height, chroma_format, slots, device=0, one_stream=False):
        self.width, self.height, self.chroma_format = width, height, chroma_format
        self.cfg = _lib.make_config(width, height, chroma_format, pool=slots, device=device,
                                    flags=_lib.MP2VG_CTX_ONE_STREAM if one_stream else 0)
        self.h = ctypes.c_void_p()
        check(lib().mp2vg_create(ctypes.byref(self.cfg), ctypes.byref(self.h)), "create")
        self.pw, self.ph, self.stride, self.slot_bytes = _lib.geometry(width, height, chroma_format)
        self.nslots = slots

    def close(self):
        if self.h:
            lib().mp2vg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, slots):
        check(lib().mp2vg_reserve_slots(self.h, slots), "reserve_slots")
        self.nslots = max(self.nslots, slots)

    def upload(self, pics, mbs, coefs):
        pics = np.ascontiguousarray(pics, PIC_DTYPE)
        mbs = np.ascontiguousarray(mbs, MB_DTYPE)
        coefs = np.ascontiguousarray(coefs, np.uint32)
        vp = ctypes.c_void_p
        check(lib().mp2vg_batch_upload(self.h, pics.ctypes.data_as(vp), len(pics), mbs.ctypes.data_as(vp), len(mbs),
                                       coefs.ctypes.data_as(vp) if len(coefs) else None, len(coefs)), "batch_upload")

    def decode(self):
        check(lib().mp2vg_batch_decode(self.h), "batch_decode")

    def synchronize(self):
        check(lib().mp2vg_synchronize(self.h), "synchronize")

    def launch_times_ms(self):
        buf = (ctypes.c_float * 256)()
        n = ctypes.c_int32()
        check(lib().mp2vg_last_launch_times(self.h, buf, 256, ctypes.byref(n)), "last_launch_times")
        return list(buf[:min(n.value, 256)])

    def batch_time_ms(self):
        """Device time of the whole last batch_decode (first launch start -> last launch end)."""
        ms = ctypes.c_float()
        check(lib().mp2vg_last_batch_time(self.h, ctypes.byref(ms)), "last_batch_time")
        return ms.value

    def batch_times(self, back=0):
        """(batch span ms, [per-launch ms]) of the batch decoded `back` decodes ago (0 = last; the
        last 64 are kept), read from the HIP events recorded when it ran."""
        ms = ctypes.c_float()
        buf = (ctypes.c_float * 256)()
        n = ctypes.c_int32()
        check(lib().mp2vg_batch_times(self.h, int(back), ctypes.byref(ms), buf, 256, ctypes.byref(n)), "batch_times")
        return ms.value, list(buf[:min(n.value, 256)])

    def batches_span(self, back_first, back_last=0):
        """Device ms from the start of the batch decoded `back_first` decodes ago to the end of the
        one `back_last` decodes ago (back-to-back batches overlap set by set)."""
        ms = ctypes.c_float()
        check(lib().mp2vg_batches_span(self.h, int(back_first), int(back_last), ctypes.byref(ms)), "batches_span")
        return ms.value

    def pool_probe(self, rw=True, reps=4):
        """Diagnostics: GB/s of each pool block (frames, tiles, frames, ... in allocation order)
        under `reps` load(+store-back) sweeps; rw=2 / 3: one rate for random / same-offset 1-KB
        reads over the pool; rw=4: per block, random 1-KB reads inside it; rw=5: the two record
        banks' MB records and coefficient words; contents kept
        (mp2vg_pool_probe)."""
        n = ctypes.c_int32()
        check(lib().mp2vg_pool_probe(self.h, int(rw), int(reps), None, 0, ctypes.byref(n)), "pool_probe")
        n.value = 1 if int(rw) in (2, 3, 6, 7) else (4 if int(rw) == 5 else n.value)
        out = np.zeros(n.value, np.float64)
        check(lib().mp2vg_pool_probe(self.h, int(rw), int(reps), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                     n.value, ctypes.byref(n)), "pool_probe")
        return out

    def placement(self):
        """The pool placement calibration of this context (mp2vg_pool_placement): (batch ms of
        each candidate pool, round 0 then round 1; index of the pool kept, -1 if it did not run)."""
        n, kept = ctypes.c_int32(), ctypes.c_int32()
        buf = (ctypes.c_float * 16)()
        check(lib().mp2vg_pool_placement(self.h, buf, 16, ctypes.byref(n), ctypes.byref(kept)), "pool_placement")
        return [round(float(v), 4) for v in buf[:min(n.value, 16)]], kept.value

    def download(self, slot):
        """Visible planes of one slot: [Y, U, V] numpy arrays (height x width)."""
        planes = [np.empty((self.ph[i], self.pw[i]), np.uint8) for i in range(3)]
        ptrs = (ctypes.c_void_p * 3)(*[p.ctypes.data for p in planes])
        check(lib().mp2vg_download_slot(self.h, slot, ptrs, None), "download_slot")
        return planes

    def frame_bytes(self):
        """Bytes of one frame in the packed write_yuv layout (Y, U, V visible planes)."""
        return sum(self.pw[i] * self.ph[i] for i in range(3))

    def copy_packed(self, slot, dst_ptr, on_device):
        """Visible planes of `slot`, packed Y|U|V, into dst_ptr (HBM of this context's device when
        on_device, e.g. a torch tensor's data_ptr(); else host memory)."""
        check(lib().mp2vg_copy_slot_packed(self.h, int(slot), ctypes.c_void_p(dst_ptr), 1 if on_device else 0),
              "copy_slot_packed")

    def digests(self, slots):
        slots = np.ascontiguousarray(slots, np.int32)
        out = np.zeros(len(slots), np.uint64)
        check(lib().mp2vg_slot_digests(self.h, slots.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(slots),
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "slot_digests")
        return out


def frame_yuv_bytes(planes):
    """The reference sample's write_yuv layout (tiny_mp2v_dec.cpp:11-17): Y, U, V rows of width."""
    return b"".join(np.ascontiguousarray(p).tobytes() for p in planes)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def planes_digest(planes):
    """Host twin of the device digest (recon.hip digest_kernel): sum over visible dwords d at
    (row_id, byte x), rows numbered across Y, U, V, of mix64(mix64((row_id << 32) | x) ^ d), mod 2^64
    (mixed after combining: paired small errors cannot cancel)."""
    total = np.uint64(0)
    row0 = 0
    with np.errstate(over="ignore"):
        for p in planes:
            p = np.ascontiguousarray(p)
            h, w = p.shape
            d = p.view("<u4").astype(np.uint64)  # (h, w/4)
            rows = (np.arange(h, dtype=np.uint64) + np.uint64(row0))[:, None]
            xs = (np.arange(w // 4, dtype=np.uint64) * np.uint64(4))[None, :]
            total = total + np.sum(_mix64(_mix64((rows << np.uint64(32)) | xs) ^ d), dtype=np.uint64)
            row0 += h
    return int(total)

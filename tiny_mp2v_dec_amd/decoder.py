"""Python mirror of the reference's public API (reference src/core/decoder.h:25-131):

    decoder_config_t{width, height, chroma_format, pictures_pool_size, num_threads, reordering}
    mp2v_decoder_c(config, renderer)   renderer(frame_c) called on a render thread, display order
    mp2v_decoder_c.decode(buf, len)    synchronous, single-shot (all frames rendered on return)
    frame_c.get_planes(i) / get_strides(i) / get_width(i) / get_height(i)

implemented over the C ABI (mp2vg_decoder_*): records are parsed on the host, reconstructed by
the HIP kernels on the GPU, and each frame is copied into a host frame with the reference's
frame_c layout before the renderer runs.  A frame is valid only during the callback (reference
frame pool recycling, threads.cpp:75-80); copy it to keep it.

decoder_config_t(devices=[0, 1, ...]) shards the stream by GOP over several GPUs
(mp2vg_decoder_create_multi: independent shards merged into runs of >= 16 pictures, run r ->
devices[r % len(devices)]); frames still reach
the renderer in display order.  After decode(), m_sequence_header / m_sequence_extension /
m_sequence_display_extension / m_group_of_pictures_header hold the stream's headers as the
reference's public members do (decoder.h:124-130).

decoder_config_t(device_frames=True) opts into the device-pointer output path
(MP2VG_DECODER_DEVICE_FRAMES): frames stay in HBM (no PCIe download), frame_c.device_ptr(i) gives
the plane's device address and get_planes(i) copies the plane to the host on demand.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib


@dataclass
class decoder_config_t:  # noqa: N801  (reference name)
    width: int
    height: int
    chroma_format: int
    pictures_pool_size: int = 10
    num_threads: int = 0
    reordering: bool = True
    device: int = 0
    device_frames: bool = False
    devices: list = None  # GOP sharding over these devices (None: [device])


MP2VG_DECODER_DEVICE_FRAMES = 1  # include/mp2vg.h
_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        else:
            raise RuntimeError("libamdhip64.so not found")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _hip


class frame_c:  # noqa: N801  (reference name)
    """View of one decoded frame (reference decoder.h:34-49)."""

    def __init__(self, f, device=False):
        self._f = f
        self.is_device = device
        self.picture_coding_type = f.picture_coding_type
        self.decode_index = f.decode_index
        self.device = f.device

    def get_planes(self, i):
        """numpy view of plane i: height x stride bytes (only valid during the callback)."""
        n = self._f.stride[i] * self._f.height[i]
        if self.is_device:  # device frame: copy the plane out of HBM (hipMemcpyDeviceToHost = 2)
            out = np.empty((self._f.height[i], self._f.stride[i]), np.uint8)
            src = ctypes.cast(self._f.planes[i], ctypes.c_void_p)
            if _hip_lib().hipMemcpy(out.ctypes.data, src, n, 2) != 0:
                raise RuntimeError("hipMemcpy of a device frame plane failed")
            return out
        return np.ctypeslib.as_array(self._f.planes[i], shape=(n,)).reshape(self._f.height[i], self._f.stride[i])

    def device_ptr(self, i):
        """Device address of plane i (device_frames decoders only; valid during the callback)."""
        if not self.is_device:
            raise ValueError("host frame: use get_planes")
        return ctypes.cast(self._f.planes[i], ctypes.c_void_p).value

    def get_strides(self, i):
        return self._f.stride[i]

    def get_width(self, i):
        return self._f.width[i]

    def get_height(self, i):
        return self._f.height[i]

    def yuv_bytes(self):
        """The reference sample's write_yuv (tiny_mp2v_dec.cpp:11-17): width bytes per row."""
        return b"".join(self.get_planes(i)[:, :self.get_width(i)].tobytes() for i in range(3))


class mp2v_decoder_c:  # noqa: N801  (reference name)
    def __init__(self, config: decoder_config_t, renderer):
        self._renderer = renderer
        self._cfg = _lib.make_config(config.width, config.height, config.chroma_format, config.pictures_pool_size,
                                     config.num_threads, config.reordering, config.device)
        self._device = bool(config.device_frames)
        self._cfg.reserved = MP2VG_DECODER_DEVICE_FRAMES if self._device else 0
        self._error = None

        def _cb(user, fptr):
            try:
                self._renderer(frame_c(fptr.contents, self._device))
            except BaseException as e:  # surface renderer errors from decode()
                if self._error is None:
                    self._error = e

        self._cb = _lib.RENDER_FN(_cb)  # keep the trampoline alive
        self._h = ctypes.c_void_p()
        devs = list(config.devices) if config.devices else [config.device]
        self._devices = devs
        arr = (ctypes.c_int32 * len(devs))(*devs)
        check(lib().mp2vg_decoder_create_multi(ctypes.byref(self._cfg), arr, len(devs), self._cb, None,
                                               ctypes.byref(self._h)), "decoder_create")
        self.user_data = []
        self.m_sequence_header = None
        self.m_sequence_extension = None
        self.m_sequence_display_extension = None
        self.m_sequence_scalable_extension = None  # scalable streams are rejected
        self.m_group_of_pictures_header = None

    def decode(self, buffer, length=None):
        data = bytes(buffer) if not isinstance(buffer, (bytes, bytearray)) else buffer
        n = len(data) if length is None else int(length)
        if n > len(data):
            raise ValueError("length exceeds the buffer")
        # no copy: the parser reads exactly [0, n) (zeros past the end, syntax.h BitReader)
        buf = np.frombuffer(data, dtype=np.uint8, count=n)
        check(lib().mp2vg_decoder_decode(self._h, buf.ctypes.data_as(ctypes.c_void_p), n), "decoder_decode")
        h = _lib.StreamHeaders()
        check(lib().mp2vg_decoder_stream_headers(self._h, ctypes.byref(h)), "decoder_stream_headers")
        self.m_sequence_header = h.sequence_header
        self.m_sequence_extension = h.sequence_extension
        self.m_sequence_display_extension = h.sequence_display_extension if h.have_sequence_display_extension else None
        self.m_group_of_pictures_header = h.group_of_pictures_header if h.have_group_of_pictures_header else None
        if self._error is not None:
            e, self._error = self._error, None
            raise e
        return True

    def flush(self, cur_pic=None):
        """reference decoder.h:100; decode() already submits and drains everything."""
        return None

    def lane_frames(self):
        """Frames each device lane decoded in the last decode() (lane i = devices[i])."""
        n = len(self._devices)
        out = (ctypes.c_int32 * n)()
        lib().mp2vg_decoder_lane_frames(self._h, out, n)
        return list(out)

    def handoff_stats(self):
        """(lane changes that left the previous lane's chunk in flight, host waits on another
        lane's downloads, lane changes whose lane just left had landed without a wait, lane
        changes) in the last decode() (mp2vg_decoder_handoff_stats)."""
        v = [ctypes.c_int32() for _ in range(4)]
        lib().mp2vg_decoder_handoff_stats(self._h, *[ctypes.byref(x) for x in v])
        return tuple(x.value for x in v)

    def frames_allocated(self):
        """Frame buffers held by the decoder's frame pools (bounded: the renderer back-pressures
        the decoder as the reference's fixed picture pool does)."""
        return lib().mp2vg_decoder_frames_allocated(self._h)

    def close(self):
        if self._h:
            lib().mp2vg_decoder_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

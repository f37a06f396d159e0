"""Python mirror of the reference's public API (reference src/core/decoder.h:25-131):

    decoder_config_t{width, height, chroma_format, pictures_pool_size, num_threads, reordering}
    mp2v_decoder_c(config, renderer)   renderer(frame_c) called on a render thread, display order
    mp2v_decoder_c.decode(buf, len)    synchronous, single-shot (all frames rendered on return)
    frame_c.get_planes(i) / get_strides(i) / get_width(i) / get_height(i)

implemented over the C ABI (mp2vg_decoder_*): records are parsed on the host, reconstructed by
the HIP kernels on the GPU, and each frame is copied into a host frame with the reference's
frame_c layout before the renderer runs.  A frame is valid only during the callback (reference
frame pool recycling, threads.cpp:75-80); copy it to keep it.
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


class frame_c:  # noqa: N801  (reference name)
    """View of one decoded frame (reference decoder.h:34-49)."""

    def __init__(self, f):
        self._f = f
        self.picture_coding_type = f.picture_coding_type
        self.decode_index = f.decode_index

    def get_planes(self, i):
        """numpy view of plane i: height x stride bytes (only valid during the callback)."""
        n = self._f.stride[i] * self._f.height[i]
        return np.ctypeslib.as_array(self._f.planes[i], shape=(n,)).reshape(self._f.height[i], self._f.stride[i])

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
        self._error = None

        def _cb(user, fptr):
            try:
                self._renderer(frame_c(fptr.contents))
            except BaseException as e:  # surface renderer errors from decode()
                if self._error is None:
                    self._error = e

        self._cb = _lib.RENDER_FN(_cb)  # keep the trampoline alive
        self._h = ctypes.c_void_p()
        check(lib().mp2vg_decoder_create(ctypes.byref(self._cfg), self._cb, None, ctypes.byref(self._h)),
              "decoder_create")

    def decode(self, buffer, length=None):
        data = bytes(buffer) if not isinstance(buffer, (bytes, bytearray)) else buffer
        n = len(data) if length is None else int(length)
        if n > len(data):
            raise ValueError("length exceeds the buffer")
        # no copy: the parser reads exactly [0, n) (zeros past the end, syntax.h BitReader)
        buf = np.frombuffer(data, dtype=np.uint8, count=n)
        check(lib().mp2vg_decoder_decode(self._h, buf.ctypes.data_as(ctypes.c_void_p), n), "decoder_decode")
        if self._error is not None:
            e, self._error = self._error, None
            raise e
        return True

    def close(self):
        if self._h:
            lib().mp2vg_decoder_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

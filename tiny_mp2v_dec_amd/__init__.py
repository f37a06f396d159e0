"""tiny_mp2v_dec_amd — MI355X-native MPEG-2 macroblock reconstruct path.

Host record emitter + HIP/CDNA4 kernels behind the C ABI of include/mp2vg.h, with the
reference's decoder API (mp2v_decoder_c / frame_c / decoder_config_t) mirrored in decoder.py.
"""
from ._lib import MB_DTYPE, PIC_DTYPE, Mp2vgError, lib  # noqa: F401
from .records import DeviceContext, Parsed, generate_es  # noqa: F401

__all__ = ["DeviceContext", "Parsed", "generate_es", "MB_DTYPE", "PIC_DTYPE", "Mp2vgError", "lib"]

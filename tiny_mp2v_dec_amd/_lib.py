"""ctypes binding of the C ABI (include/mp2vg.h) and numpy views of the record stream.

The native library is REQUIRED: there is no Python or CPU fallback for the reconstruct path.
Loading fails loudly when libmp2vg.so is missing (run tiny_mp2v_dec_amd/build.py).
"""
import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MP2VG_LIB") or os.path.join(PKG, "_build", "libmp2vg.so")  # override: dev A/B builds

# ---- record dtypes (must match include/mp2vg.h) ------------------------------------------
MB_DTYPE = np.dtype([("x", "<u2"), ("y", "<u2"), ("flags", "<u2"), ("cbp", "<u2"), ("qscale", "u1"),
                     ("reserved", "u1"), ("ncoef", "<u2"), ("coef_off", "<u4"), ("mv", "<i2", (2, 2, 2))])
assert MB_DTYPE.itemsize == 32
PIC_DTYPE = np.dtype([("dst_slot", "<i4"), ("fwd_slot", "<i4"), ("bwd_slot", "<i4"),
                      ("picture_coding_type", "<i4"), ("mb_first", "<u4"), ("mb_width", "<u2"),
                      ("mb_height", "<u2"), ("alternate_scan", "u1"), ("reserved0", "u1", (3,)),
                      ("temporal_reference", "<i4"), ("W", "u1", (4, 64))])
assert PIC_DTYPE.itemsize == 288

MB_INTRA, MB_FWD, MB_BWD, MB_FIELD_MC, MB_DCT_FIELD = 1, 2, 4, 8, 16
COEF_FIRST1S, COEF_DC = 1 << 29, 1 << 30


def mb_fs_bit(r, s):
    return 1 << (8 + 2 * r + s)


def coef_pack(level, pos, block, flags=0, mbx=0):
    """Coefficient word (include/mp2vg.h); mbx = the MB's column (bits 26-28 carry mbx & 7)."""
    return (np.uint32(np.int64(level) & 0xFFFF) | np.uint32(pos << 16) | np.uint32(block << 22) |
            np.uint32(flags) | np.uint32((int(mbx) & 7) << 26))


STATUS = {0: "ok", -1: "invalid argument", -2: "unsupported stream", -3: "HIP error", -4: "out of memory",
          -5: "call out of order", -6: "bitstream error"}


class Mp2vgError(RuntimeError):
    def __init__(self, status, what, detail=""):
        self.status = status
        super().__init__(f"{what}: {STATUS.get(status, status)} ({detail})")


class Config(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("chroma_format", ctypes.c_int32),
                ("pictures_pool_size", ctypes.c_int32), ("num_threads", ctypes.c_int32),
                ("reordering", ctypes.c_int32), ("device", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class GenParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "width", "height", "chroma_format", "n_gops", "gop_n", "gop_m")] + [("seed", ctypes.c_uint32)] + [
        (n, ctypes.c_int32) for n in (
            "frame_pred_frame_dct", "alternate_scan", "q_scale_type", "intra_dc_precision", "coefs_min",
            "coefs_max", "intra_coefs_min", "intra_coefs_max", "big_level_permille", "escape_permille",
            "quant_permille", "f_code", "mix", "leading_b", "big_matrix_permille")] + [
        ("reserved", ctypes.c_int32 * 5)]


class Frame(ctypes.Structure):
    _fields_ = [("planes", ctypes.POINTER(ctypes.c_uint8) * 3), ("width", ctypes.c_int32 * 3),
                ("height", ctypes.c_int32 * 3), ("stride", ctypes.c_int32 * 3),
                ("picture_coding_type", ctypes.c_int32), ("decode_index", ctypes.c_int32),
                ("device", ctypes.c_int32)]


class SequenceHeader(ctypes.Structure):  # mp2vg_sequence_header_t (reference mp2v_hdr.h:61-75)
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "sequence_header_code", "horizontal_size_value", "vertical_size_value", "aspect_ratio_information",
        "frame_rate_code", "bit_rate_value", "vbv_buffer_size_value", "constrained_parameters_flag",
        "load_intra_quantiser_matrix")] + [("intra_quantiser_matrix", ctypes.c_uint8 * 64),
                                           ("load_non_intra_quantiser_matrix", ctypes.c_uint32),
                                           ("non_intra_quantiser_matrix", ctypes.c_uint8 * 64)]


class SequenceExtension(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "extension_start_code", "extension_start_code_identifier", "profile_and_level_indication",
        "progressive_sequence", "chroma_format", "horizontal_size_extension", "vertical_size_extension",
        "bit_rate_extension", "vbv_buffer_size_extension", "low_delay", "frame_rate_extension_n",
        "frame_rate_extension_d")]


class SequenceDisplayExtension(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "extension_start_code_identifier", "video_format", "colour_description", "colour_primaries",
        "transfer_characteristics", "matrix_coefficients", "display_horizontal_size", "display_vertical_size")]


class GopHeader(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("group_start_code", "time_code", "closed_gop", "broken_link")]


class StreamHeaders(ctypes.Structure):  # mp2vg_stream_headers_t
    _fields_ = [("have_sequence_display_extension", ctypes.c_int32),
                ("have_group_of_pictures_header", ctypes.c_int32),
                ("sequence_header", SequenceHeader), ("sequence_extension", SequenceExtension),
                ("sequence_display_extension", SequenceDisplayExtension),
                ("group_of_pictures_header", GopHeader)]


RENDER_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(Frame))

# every symbol declared in include/mp2vg.h
EXPORTS = [
    "mp2vg_abi_version", "mp2vg_status_string", "mp2vg_last_error", "mp2vg_create", "mp2vg_destroy",
    "mp2vg_frame_geometry", "mp2vg_reserve_slots", "mp2vg_batch_upload", "mp2vg_batch_validate", "mp2vg_batch_decode",
    "mp2vg_synchronize", "mp2vg_last_launch_times", "mp2vg_last_batch_time", "mp2vg_batch_times", "mp2vg_batches_span", "mp2vg_download_slot", "mp2vg_copy_slot_packed", "mp2vg_slot_device_ptr", "mp2vg_sink_device_ptr", "mp2vg_clock_probe", "mp2vg_pool_probe", "mp2vg_pool_placement", "mp2vg_cpu_budget", "mp2vg_invalidate_slot",
    "mp2vg_slot_digests", "mp2vg_parse_es", "mp2vg_parsed_counts", "mp2vg_parsed_pictures", "mp2vg_parsed_mbs",
    "mp2vg_parsed_coefs", "mp2vg_parsed_display_order", "mp2vg_parsed_gop_index", "mp2vg_parsed_stream_headers",
    "mp2vg_parsed_shards", "mp2vg_parsed_free", "mp2vg_vlc_decode",
    "mp2vg_gen_default_params", "mp2vg_generate_es", "mp2vg_free", "mp2vg_decoder_create",
    "mp2vg_decoder_create_multi", "mp2vg_decoder_decode", "mp2vg_decoder_stream_headers",
    "mp2vg_decoder_lane_frames", "mp2vg_decoder_frames_allocated", "mp2vg_decoder_handoff_stats",
    "mp2vg_decoder_destroy",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"native library {LIB_PATH} is missing: run `python tiny_mp2v_dec_amd/build.py` "
                           "(there is no CPU fallback for the reconstruct path)")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, U64, VP = ctypes.POINTER, ctypes.c_int32, ctypes.c_uint64, ctypes.c_void_p
    sig = {
        "mp2vg_abi_version": ([], ctypes.c_int),
        "mp2vg_status_string": ([ctypes.c_int], ctypes.c_char_p),
        "mp2vg_last_error": ([], ctypes.c_char_p),
        "mp2vg_create": ([P(Config), P(VP)], ctypes.c_int),
        "mp2vg_destroy": ([VP], ctypes.c_int),
        "mp2vg_frame_geometry": ([P(Config), P(I32), P(I32), P(I32), P(U64)], ctypes.c_int),
        "mp2vg_reserve_slots": ([VP, I32], ctypes.c_int),
        "mp2vg_batch_upload": ([VP, VP, I32, VP, U64, VP, U64], ctypes.c_int),
        "mp2vg_batch_validate": ([P(Config), I32, VP, I32, VP, U64, VP, U64, P(I32), P(I32), P(I32), I32],
                                 ctypes.c_int),
        "mp2vg_batch_decode": ([VP], ctypes.c_int),
        "mp2vg_synchronize": ([VP], ctypes.c_int),
        "mp2vg_last_launch_times": ([VP, P(ctypes.c_float), I32, P(I32)], ctypes.c_int),
        "mp2vg_last_batch_time": ([VP, P(ctypes.c_float)], ctypes.c_int),
        "mp2vg_batch_times": ([VP, I32, P(ctypes.c_float), P(ctypes.c_float), I32, P(I32)], ctypes.c_int),
        "mp2vg_batches_span": ([VP, I32, I32, P(ctypes.c_float)], ctypes.c_int),
        "mp2vg_download_slot": ([VP, I32, P(ctypes.c_void_p), P(I32)], ctypes.c_int),
        "mp2vg_copy_slot_packed": ([VP, I32, VP, I32], ctypes.c_int),
        "mp2vg_slot_device_ptr": ([VP, I32, P(VP)], ctypes.c_int),
        "mp2vg_sink_device_ptr": ([VP, P(VP)], ctypes.c_int),
        "mp2vg_clock_probe": ([I32, P(ctypes.c_double)], ctypes.c_int),
        "mp2vg_pool_probe": ([VP, I32, I32, P(ctypes.c_double), I32, P(I32)], ctypes.c_int),
        "mp2vg_pool_placement": ([VP, P(ctypes.c_float), I32, P(I32), P(I32)], ctypes.c_int),
        "mp2vg_cpu_budget": ([], ctypes.c_int),
        "mp2vg_invalidate_slot": ([VP, I32], ctypes.c_int),
        "mp2vg_slot_digests": ([VP, P(I32), I32, P(ctypes.c_uint64)], ctypes.c_int),
        "mp2vg_parse_es": ([VP, U64, P(Config), P(VP)], ctypes.c_int),
        "mp2vg_parsed_counts": ([VP, P(I32), P(U64), P(U64)], ctypes.c_int),
        "mp2vg_parsed_pictures": ([VP], VP),
        "mp2vg_parsed_mbs": ([VP], VP),
        "mp2vg_parsed_coefs": ([VP], VP),
        "mp2vg_parsed_display_order": ([VP, P(I32), I32], ctypes.c_int),
        "mp2vg_parsed_gop_index": ([VP, P(I32), I32], ctypes.c_int),
        "mp2vg_parsed_stream_headers": ([VP, P(StreamHeaders)], ctypes.c_int),
        "mp2vg_parsed_shards": ([VP, P(I32), I32], ctypes.c_int),
        "mp2vg_parsed_free": ([VP], None),
        "mp2vg_vlc_decode": ([I32, U64, P(I32), P(I32), P(I32)], ctypes.c_int),
        "mp2vg_gen_default_params": ([P(GenParams)], None),
        "mp2vg_generate_es": ([P(GenParams), P(VP), P(U64)], ctypes.c_int),
        "mp2vg_free": ([VP], None),
        "mp2vg_decoder_create": ([P(Config), RENDER_FN, VP, P(VP)], ctypes.c_int),
        "mp2vg_decoder_create_multi": ([P(Config), P(I32), I32, RENDER_FN, VP, P(VP)], ctypes.c_int),
        "mp2vg_decoder_decode": ([VP, VP, U64], ctypes.c_int),
        "mp2vg_decoder_stream_headers": ([VP, P(StreamHeaders)], ctypes.c_int),
        "mp2vg_decoder_lane_frames": ([VP, P(I32), I32], ctypes.c_int),
        "mp2vg_decoder_frames_allocated": ([VP], ctypes.c_int),
        "mp2vg_decoder_handoff_stats": ([VP, P(I32), P(I32), P(I32), P(I32)], ctypes.c_int),
        "mp2vg_decoder_destroy": ([VP], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(status, what):
    if status != 0:
        detail = lib().mp2vg_last_error().decode(errors="replace")
        raise Mp2vgError(status, what, detail)
    return status


MP2VG_DECODER_DEVICE_FRAMES, MP2VG_CTX_ONE_STREAM = 1, 2  # mp2vg_config_t.reserved flags


def make_config(width, height, chroma_format, pool=10, threads=0, reordering=True, device=0, flags=0):
    return Config(width, height, chroma_format, pool, threads, 1 if reordering else 0, device, flags)


def geometry(width, height, chroma_format):
    c = make_config(width, height, chroma_format)
    w, h, s = (ctypes.c_int32 * 3)(), (ctypes.c_int32 * 3)(), (ctypes.c_int32 * 3)()
    sb = ctypes.c_uint64()
    check(lib().mp2vg_frame_geometry(ctypes.byref(c), w, h, s, ctypes.byref(sb)), "frame_geometry")
    return list(w), list(h), list(s), sb.value

"""ctypes binding of the C oracle (oracle/build/liboracle.so) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker (see oracle/mp2v_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")


class Geom(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("chroma_format", ctypes.c_int),
                ("pw", ctypes.c_int * 3), ("ph", ctypes.c_int * 3), ("stride", ctypes.c_int * 3),
                ("plane_off", ctypes.c_uint64 * 3), ("slot_bytes", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "build/liboracle.so"])
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_geometry.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Geom)]
        L.oracle_reconstruct.argtypes = [ctypes.POINTER(Geom), ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_reconstruct.restype = ctypes.c_int
        L.oracle_idct.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_mc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_dequant_block.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


def geometry(width, height, chroma_format):
    g = Geom()
    lib().oracle_geometry(width, height, chroma_format, ctypes.byref(g))
    return g


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def idct(F, pred=None):
    """F: int16[64] (QFS layout).  Returns 8x8 uint8 put (pred None) or add over pred."""
    F = np.ascontiguousarray(F, dtype=np.int16)
    out = np.zeros(64, np.uint8) if pred is None else np.array(pred, dtype=np.uint8).copy()
    lib().oracle_idct(_ptr(F), _ptr(out), 8, 0 if pred is None else 1)
    return out


def mc(dst, src0, off0, src1, off1, stride, width, height, bidir, idx):
    base0 = src0.ctypes.data + off0
    base1 = (src1.ctypes.data + off1) if src1 is not None else None
    lib().oracle_mc(_ptr(dst), ctypes.c_void_p(base0), ctypes.c_void_p(base1) if base1 else None,
                    stride, width, height, bidir, idx)


def reconstruct(width, height, chroma_format, pics, mbs, coefs, nslots):
    """pics/mbs/coefs: numpy structured arrays / uint32 array (tiny_mp2v_dec_amd.records dtypes)."""
    g = geometry(width, height, chroma_format)
    pool = np.zeros(int(g.slot_bytes) * nslots + 64, np.uint8)
    rc = lib().oracle_reconstruct(ctypes.byref(g), _ptr(pics), len(pics), _ptr(mbs), _ptr(coefs),
                                  _ptr(pool), nslots)
    if rc != 0:
        raise RuntimeError("oracle_reconstruct failed")
    return g, pool

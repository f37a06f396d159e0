"""CPU: the C-ABI library loads, exports exactly what include/*.h declares, and fails loudly (no
CPU fallback) when device work is requested without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from tiny_mp2v_dec_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(REPO, "include", "mp2vg.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mp2vg_[a-z_0-9]+)\s*\(", text)) - {"mp2vg_mb", "mp2vg_picture"})


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_every_declared_symbol_exported():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (mp2vg_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    """The embedded HIP fat binary carries a gfx950 code object (and no other target)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}


def test_abi_version_and_status_strings():
    L = _lib.lib()
    assert L.mp2vg_abi_version() == 2  # 2: coefficient-word bit layout of round 2
    for s in (0, -1, -2, -3, -4, -5, -6):
        assert L.mp2vg_status_string(s)


def test_struct_layouts():
    assert _lib.MB_DTYPE.itemsize == 32
    assert _lib.PIC_DTYPE.itemsize == 288
    assert ctypes.sizeof(_lib.Config) == 32


def test_frame_geometry_matches_reference_frame_c():
    """frame_c (reference decoder.cpp:44-68): stride = round_up(w, 64); chroma = round_up(stride/2, 64)"""
    w, h, s, slot = _lib.geometry(1920, 1088, 1)
    assert (w, h, s) == ([1920, 960, 960], [1088, 544, 544], [1920, 960, 960])
    assert slot == 1920 * 1088 + 2 * 960 * 544
    w, h, s, _ = _lib.geometry(176, 144, 2)
    assert (w, h, s) == ([176, 88, 88], [144, 144, 144], [192, 128, 128])
    w, h, s, _ = _lib.geometry(3840, 2160 + 16 - 2160 % 16, 3)
    assert s == [3840, 3840, 3840]
    with pytest.raises(_lib.Mp2vgError):
        _lib.geometry(100, 64, 1)


def test_invalid_arguments_rejected():
    L = _lib.lib()
    assert L.mp2vg_create(None, None) == -1
    assert L.mp2vg_batch_decode(None) == -1
    assert L.mp2vg_destroy(None) == -1
    n = ctypes.c_int32()
    assert L.mp2vg_pool_probe(None, 1, 1, None, 0, ctypes.byref(n)) == -1
    assert L.mp2vg_clock_probe(0, None) == -1
    assert L.mp2vg_sink_device_ptr(None, None) == -1


def test_no_silent_cpu_fallback_without_gpu():
    """Without a device the context cannot be created: the product path has no CPU fallback."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    cfg = _lib.make_config(176, 144, 1)
    h = ctypes.c_void_p()
    rc = _lib.lib().mp2vg_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == -3  # MP2VG_E_HIP


def test_cpu_budget_within_the_process_cpus():
    """mp2vg_cpu_budget (the decoder's default thread count): at least 1, at most the CPUs this
    process may run on, and at most a cgroup v2 cpu.max quota when one is set."""
    import os
    n = _lib.lib().mp2vg_cpu_budget()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            assert n <= max(1, int(q) // int(period))
    except (OSError, ValueError):
        pass

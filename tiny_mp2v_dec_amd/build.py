"""Build the native library in-tree: tiny_mp2v_dec_amd/_build/libmp2vg.so (hipcc, gfx950 only).

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.  Incremental: an
object is rebuilt when its source or any csrc/ header / include/ header is newer.
"""
import concurrent.futures
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_build")
LIB = os.path.join(OUT, "libmp2vg.so")
CLI = os.path.join(OUT, "tiny_mp2v_dec_gpu")
ARCH = os.environ.get("MP2VG_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj):
    hipcc = _hipcc()
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-I", CSRC, "-I", os.path.join(REPO, "include")]
    if src.endswith(".hip"):
        cmd = [hipcc, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + common + ["-c", src, "-o", obj]
    else:
        # host translation units (HIP runtime API only): compiled as host C++ by hipcc
        cmd = [hipcc, "-D__HIP_PLATFORM_AMD__"] + common + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False):
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = _headers()
    jobs = []
    objs = []
    # a library newer than every source and header is current even when its objects are absent
    # (they are gpurun-ignored, so the GPU box gets the .so alone)
    lib_current = not _stale(LIB, srcs + hdrs)
    for s in srcs:
        if lib_current:
            break
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(o, [s] + hdrs):
            jobs.append((s, o))
    if jobs:
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            for o in ex.map(lambda j: _compile(*j), jobs):
                if verbose:
                    print("built", os.path.relpath(o, REPO))
    if not lib_current and _stale(LIB, objs):
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("linked", os.path.relpath(LIB, REPO))
    # the reference CLI sample rebuilt against the drop-in header (include/mp2v_decoder.h)
    cli_src = os.path.join(REPO, "tools", "tiny_mp2v_dec_gpu.cpp")
    if os.path.exists(cli_src) and _stale(CLI, [cli_src, LIB] + hdrs):
        cmd = ["g++", "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"), cli_src, "-o", CLI, "-L", OUT,
               "-lmp2vg", "-Wl,-rpath,$ORIGIN"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"cli build failed: {' '.join(cmd)}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    print(LIB)
    sys.exit(0)

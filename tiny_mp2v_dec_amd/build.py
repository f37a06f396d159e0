"""Build the native library in-tree: tiny_mp2v_dec_amd/_build/libmp2vg.so (hipcc, gfx950 only).

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.  Provenance is by
content, not mtime: libmp2vg.so.stamp holds a SHA-256 over every source and header, the target
arch and every compile / link command.  The library is current exactly when its stamp matches
(so the GPU box, which gets the .so without objects, rebuilds nothing, and a change of
MP2VG_OFFLOAD_ARCH or flags always rebuilds); each object carries the same kind of stamp.
"""
import concurrent.futures
import glob
import hashlib
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


def _digest(files, cmds):
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    for c in cmds:  # tool by name, in-tree paths relative to the repo (the GPU box's copy lives elsewhere)
        h.update("\0".join(os.path.basename(x) if x == c[0] else x.replace(REPO, "<repo>") for x in c).encode()
                 + b"\n")
    return h.hexdigest()


def _current(target, stamp):
    try:
        with open(target + ".stamp") as fh:
            return os.path.exists(target) and fh.read().strip() == stamp
    except OSError:
        return False


def _write_stamp(target, stamp):
    with open(target + ".stamp", "w") as fh:
        fh.write(stamp + "\n")


def _compile_cmd(src, obj):
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-I", CSRC, "-I", os.path.join(REPO, "include")]
    if src.endswith(".hip"):
        return [_hipcc(), "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + common + ["-c", src, "-o", obj]
    # host translation units (HIP runtime API only): compiled as host C++ by hipcc
    return [_hipcc(), "-D__HIP_PLATFORM_AMD__"] + common + ["-c", src, "-o", obj]


def _compile(src, obj, stamp):
    cmd = _compile_cmd(src, obj)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    _write_stamp(obj, stamp)
    return obj


def _git_head():
    """`git rev-parse HEAD` (+ "-dirty" when tracked files differ), or None without a checkout."""
    try:
        head = subprocess.run(["git", "-C", REPO, "rev-parse", "HEAD"], capture_output=True, text=True,
                              timeout=20).stdout.strip()
        if not head:
            return None
        dirty = subprocess.run(["git", "-C", REPO, "status", "--porcelain", "--untracked-files=no"],
                               capture_output=True, text=True, timeout=20).stdout.strip()
        return head + ("-dirty" if dirty else "")
    except (OSError, subprocess.SubprocessError):
        return None


def provenance():
    """What a log or bench line ran: the git commit (live in a checkout; on the GPU box, which gets
    the tree without .git, the commit build() recorded in _build/HEAD) and the library's content
    stamp (a SHA-256 over every source, header and build command: recomputable from any commit)."""
    try:
        with open(LIB + ".stamp") as fh:
            stamp = fh.read().strip()
    except OSError:
        stamp = None
    head = _git_head()
    src = "git"
    verified = None
    if head is None:
        # _build/HEAD: line 1 the commit, line 2 the library stamp build() produced at that commit.
        # The head is vouched for only while the library loaded now is that same build
        try:
            with open(os.path.join(OUT, "HEAD")) as fh:
                lines = fh.read().split()
            head, src = (lines[0] if lines else None), "_build/HEAD (recorded by build())"
            verified = len(lines) > 1 and stamp is not None and lines[1] == stamp
        except OSError:
            src = None
    out = {"head": head, "head_source": src, "libmp2vg_stamp": stamp}
    if verified is not None:
        out["head_matches_library"] = verified
    return out


def build(verbose=False):
    os.makedirs(OUT, exist_ok=True)
    head = _git_head()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = _headers()
    objs = [os.path.join(OUT, os.path.basename(s) + ".o") for s in srcs]
    link_cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lpthread"]
    lib_stamp = _digest(srcs + hdrs, [_compile_cmd(s, o) for s, o in zip(srcs, objs)] + [link_cmd])
    if not _current(LIB, lib_stamp):
        jobs = []
        for s, o in zip(srcs, objs):
            st = _digest([s] + hdrs, [_compile_cmd(s, o)])
            if not _current(o, st):
                jobs.append((s, o, st))
        if jobs:
            with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
                for o in ex.map(lambda j: _compile(*j), jobs):
                    if verbose:
                        print("built", os.path.relpath(o, REPO))
        r = subprocess.run(link_cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(link_cmd)}\n{r.stdout}\n{r.stderr}")
        _write_stamp(LIB, lib_stamp)
        if verbose:
            print("linked", os.path.relpath(LIB, REPO))
    if head is not None:  # the commit, and the library build() produced at it (provenance())
        with open(os.path.join(OUT, "HEAD"), "w") as fh:
            fh.write(f"{head}\n{lib_stamp}\n")
    # the reference CLI sample rebuilt against the drop-in header (include/mp2v_decoder.h)
    cli_src = os.path.join(REPO, "tools", "tiny_mp2v_dec_gpu.cpp")
    if os.path.exists(cli_src):
        cmd = ["g++", "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"), cli_src, "-o", CLI, "-L", OUT,
               "-lmp2vg", "-Wl,-rpath,$ORIGIN"]
        st = _digest([cli_src] + hdrs, [cmd]) + lib_stamp
        if not _current(CLI, st):
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"cli build failed: {' '.join(cmd)}\n{r.stderr}")
            _write_stamp(CLI, st)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    print(LIB)
    sys.exit(0)

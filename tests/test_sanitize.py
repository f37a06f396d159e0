"""CPU: the host code that consumes untrusted input, built with AddressSanitizer and
UndefinedBehaviorSanitizer, survives mutated streams and corrupted record batches.

tests/fuzz/parse_fuzz.cpp is compiled with g++ -fsanitize=address,undefined together with the
record emitter (parse.cpp, tables.cpp) and the upload validation (runtime.cpp's
mp2vg_batch_validate, no device needed).  Over the golden streams it feeds bit flips, random
spans, truncations, deleted / duplicated spans and injected start codes to the whole-stream
parse and to the drop-in's streaming parse session, and records with corrupted fields to the
validation.  Rejections are expected; any out-of-bounds access, leak or undefined behaviour
aborts the harness (-fno-sanitize-recover=all) and fails the test.  The records of every mutant
that parses must pass the full upload validation unmodified: the drop-in uploads the parser's
records on the trusted path, so the parser itself has to uphold every invariant the kernels rely
on.  Findings so far, fixed:
a zero-picture stream passed a null pointer to memcpy, and f_code = 0 made the motion-vector
parse read -1 bits (now rejected like the reference's undefined read)."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "tiny_mp2v_dec_amd", "csrc")
STREAMS = os.path.join(REPO, "tests", "golden", "streams")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("san") / "parse_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-w", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-DWITH_VALIDATE", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
           "-I", CSRC, "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "fuzz", "parse_fuzz.cpp"),
           os.path.join(CSRC, "parse.cpp"), os.path.join(CSRC, "tables.cpp"), os.path.join(CSRC, "runtime.cpp"),
           "-o", exe, "-pthread", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(f"sanitizer build failed:\n{r.stderr[-2000:]}")
    return exe


def _args(names):
    man = {m["name"]: m for m in json.load(open(os.path.join(STREAMS, "manifest.json")))}
    out = []
    for n in names:
        m = man[n]
        out += [os.path.join(STREAMS, m["file"]), str(m["width"]), str(m["height"]), str(m["chroma_format"])]
    return out


@pytest.mark.parametrize("names,seed", [
    (["ipb420_qcif", "ipb420_field", "ipb422_field", "ipb444_field"], 1),
    (["stress_saturation", "stress_mv_fcode4", "mc_heavy_fcode1", "ipb420_qcif_openb"], 2),
    (["i420_cif_intra", "ipb422_qcif", "ipb444_qcif", "tall_2816_vpos_ext"], 3),
])
def test_mutated_streams_under_asan_ubsan(harness, names, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, "120", str(seed)] + _args(names), capture_output=True, text=True, timeout=900,
                       env=env)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-3000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mutants_rejected"] > 0 and res["batches_rejected"] > 0 and res["batches_valid"] > 0


@pytest.fixture(scope="module")
def tsan_harness(tmp_path_factory):
    """The same harness under ThreadSanitizer: every slice is a parse task, so the slices of one
    picture run on several workers and publish the picture through an atomic countdown."""
    exe = str(tmp_path_factory.mktemp("tsan") / "parse_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-w", "-fsanitize=thread", "-fno-omit-frame-pointer",
           "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include", "-I", CSRC, "-I", os.path.join(REPO, "include"),
           os.path.join(REPO, "tests", "fuzz", "parse_fuzz.cpp"), os.path.join(CSRC, "parse.cpp"),
           os.path.join(CSRC, "tables.cpp"), "-o", exe, "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"ThreadSanitizer build unavailable:\n{r.stderr[-800:]}")
    return exe


def test_slice_parallel_parse_under_tsan(tsan_harness):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([tsan_harness, "25", "4"] + _args(["hd1080_420_ipb", "ipb420_field", "ipb444_qcif",
                                                          "stress_saturation"]),
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-3000:])
    assert "WARNING: ThreadSanitizer" not in r.stderr

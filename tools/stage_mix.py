"""Static instruction mix per loop stage of a recon kernel, priced with measured issue costs (dev tool).

    python tools/stage_mix.py [--kernel 1,2] [--asm out.s]

Compiles recon.hip's stamp build (-DMP2VG_DEV_ABLATIONS, ABL 16: an s_memtime at each stage
boundary of the loop, tools/stamps.py) to gfx950 assembly, walks the loop body (blocks inside
the group loop) in layout order, splits it at the s_memtime markers and counts per stage:
  fast VALU   v_add/v_sub/v_and/v_or/v_xor/v_mov/v_lshrrev/v_ashrrev/v_add_u16 with VGPR, inline or
              literal operands: 1.68 SIMD cycles per wave64 instruction at 4 waves per SIMD
  slow VALU   every other VALU form (v_lshlrev, multiplies, 3-operand VOP3, VOP3P, SDWA, DPP,
              cndmask_e64, a VOP2 with an SGPR operand): 2.68-2.74 cycles
  LDS, ds_bpermute/ds_swizzle, VMEM, SALU, branches, s_waitcnt (counts only)
The costs are tools/issue_bench.hip's (profiles/r6/issue_bench.txt).  Blocks of inner loops (IDCT
rounds, dequant word rounds) count once: a B/P group runs about one round of each.  The model
cycles per stage are VALU only (fast x 1.68 + slow x 2.74): compare with the stage's measured
cycles (tools/stamps.py) to see which stages issue at the VALU rate and which wait.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32", "v_lshrrev_b32",
        "v_ashrrev_i32", "v_add_u16", "v_sub_u16"}
COST = {"fast": 1.68, "slow": 2.74}
STAGES = ["wait taps + predict", "look-ahead issue", "dequant", "idct pass 1 + chroma issue", "idct pass 2",
          "add/clip + store", "latch"]


def classify(m, ops):
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", m)
    if m.startswith("v_"):
        if m.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "vlane"
        if base in FAST and not m.endswith(("_sdwa", "_dpp")) and not re.search(r"(^|[\s,])s\d|s\[", ops) \
                and "vcc" not in ops.split(",")[0]:
            return "fast"
        return "slow"
    if m.startswith(("ds_bpermute", "ds_permute", "ds_swizzle")):
        return "xlane"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if m.startswith("s_waitcnt"):
        return "wait"
    if m.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if m.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="1,2", help="chroma format, mc mode")
    ap.add_argument("--asm", default="/tmp/stage_mix.s")
    ap.add_argument("--src", default=os.path.join(REPO, "tiny_mp2v_dec_amd", "csrc", "recon.hip"))
    a = ap.parse_args()
    cf, mcm = a.kernel.split(",")
    cmd = ["hipcc", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-O3", "-std=c++17",
           "-DMP2VG_DEV_ABLATIONS", "-I", os.path.join(REPO, "tiny_mp2v_dec_amd", "csrc"), "-I", os.path.join(REPO, "include"),
           a.src, "-o", a.asm]
    subprocess.run(cmd, check=True, capture_output=True)
    lines = open(a.asm).read().split("\n")
    sym = f"_ZN5mp2vg12recon_kernelILi{cf}ELi{mcm}ELi16E"
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and ":" in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    depth = 0
    stage = None
    per = collections.defaultdict(collections.Counter)
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2))
            depth = int(d.group(1)) if d else 0
            continue
        t = l.strip()
        ms = re.search(r"s_memtime .*stage stamp (-?\d+)", t)
        if ms:
            # stamp i closes stage i (6: the latch, taken at the loop top); the code after it
            # belongs to the stage the next stamp closes: 6 -> 0 -> 1 ... -> 5 -> 6
            i = int(ms.group(1))
            stage = 0 if i in (-1, 6) else i + 1
            continue
        if not t or t.startswith((";", ".", "@")) or t.endswith(":"):
            continue
        parts = t.split(None, 1)
        mn, ops = parts[0], parts[1] if len(parts) > 1 else ""
        if depth >= 1 and stage is not None:
            per[stage][classify(mn, ops)] += 1
    cols = ["fast", "slow", "vlane", "lds", "xlane", "vmem", "salu", "branch", "wait"]
    print(f"recon_kernel<{cf},{mcm}> loop, static per stage (inner-loop bodies once)\n")
    print("| stage | " + " | ".join(cols) + " | VALU model cycles |")
    print("|---|" + "---|" * (len(cols) + 1))
    tot = collections.Counter()
    for s in range(len(STAGES)):
        c = per[s]
        tot.update(c)
        model = c["fast"] * COST["fast"] + (c["slow"] + c["vlane"]) * COST["slow"]
        name = STAGES[s]
        print(f"| {name} | " + " | ".join(str(c[k]) for k in cols) + f" | {model:.0f} |")
    model = tot["fast"] * COST["fast"] + (tot["slow"] + tot["vlane"]) * COST["slow"]
    print("| total | " + " | ".join(str(tot[k]) for k in cols) + f" | {model:.0f} |")


if __name__ == "__main__":
    sys.exit(main())

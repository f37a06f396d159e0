"""Static VALU issue-cost estimate of a kernel's main loop from hipcc -S output (dev tool).

    python tools/isa_cost.py <file.s> <kernel symbol substring>

Weights per wave-instruction per SIMD are the gfx950 rates measured by tools/valu_bench.hip:
VOP1/VOP2 (e32, sdwa) 2.3, VOP3/VOP3P 4.5, v_mul_lo/v_mul_hi 9, DPP 4.4; LDS and memory ops are
counted separately (they issue to other pipes).  Inner loops (IDCT passes, rare coefficient
loop) are reported per block so their trip counts can be applied by hand.
"""
import re
import sys
from collections import Counter, OrderedDict


def cost(ins, ops):
    if ins.startswith(("v_mul_lo_u32", "v_mul_hi", "v_mad_u64", "v_mad_i64")):
        return 9.0
    if ins.startswith("v_pk_") or ins.endswith("_e64") or "dpp" in ops:
        return 4.5
    if ins.endswith("_e32") or ins.endswith("_sdwa"):
        return 2.3
    if ins.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return 2.3
    if ins.startswith("v_"):
        return 4.5  # VOP3-only encodings: perm, alignbyte, lerp, bfe, add3, lshl_add, cndmask (3 src), ...
    return 0.0


def main(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or (sym in l and l.endswith(": ; @" + l.split(":")[0])))
    body = []
    for l in lines[start + 1:]:
        if "s_endpgm" in l:
            break
        body.append(l)
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in body:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            tag = l.split(";", 1)[1].strip() if ";" in l else ""
            blocks[cur].append(("#", tag))
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        parts = t.split(None, 1)
        blocks[cur].append((parts[0], parts[1] if len(parts) > 1 else ""))
    for name, ins in blocks.items():
        tag = ins[0][1] if ins and ins[0][0] == "#" else ""
        c = sum(cost(i, o) for i, o in ins if i != "#")
        n_valu = sum(1 for i, o in ins if i.startswith("v_"))
        lds = sum(1 for i, o in ins if i.startswith("ds_"))
        vmem = sum(1 for i, o in ins if i.startswith(("buffer_", "global_", "scratch_")))
        if n_valu or lds or vmem:
            print(f"{name:12s} valu {n_valu:4d} cyc {c:7.1f} lds {lds:3d} vmem {vmem:3d}  {tag[:60]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

"""Line-granular floor of the P/B reconstruct kernels' memory pipeline (dev analysis).

For a bench batch (default: c2, 8 GOPs of the seed-1729 stream; scaled to the bench's GOPs per
step) this replays, on the host, every vector-memory wave-instruction the P/B kernels issue for
reference taps and row stores under today's lane mapping (recon.hip: one lane = one pixel row of
one MB, 4 MBs per wave group; luma b128 + b32 per row and direction, second half-pel rows only on
the MB's edge lanes; 4:2:0 chroma b96 per Cb / Cr row; 16-B luma and 8-B chroma row stores), and
counts

  * TA lookups: distinct 128-B lines (and 64-B sectors) per wave-instruction, summed;
  * group lines: distinct 128-B lines per 4-MB group over all its instructions -- what the L1
    must fetch from L2 for the group if nothing is reused across groups;
  * the same two counts under alternative layouts of the anchor pictures (the taps' source):
      tile8x16  -- 128-B tiles of 8 rows x 16 px (no apron: a 17-px row spans two tiles, two
                   loads per row)
      apron4x32 -- 128-B tiles of 4 rows x 32 B (16 px + a 16-px apron: one load per row)
      (chroma: 8 rows x 16 B tiles, 8 px + 8-px apron, in both).

  python tools/line_floor.py [config] [gops] [--json out.json]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from tiny_mp2v_dec_amd import _lib  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

MB_INTRA, MB_FWD, MB_BWD, MB_FIELD_MC = 1, 2, 4, 8


def count_unique(ids, lines):
    """Distinct (instruction id, line) pairs and distinct instruction ids."""
    key = ids.astype(np.int64) * (1 << 34) + lines.astype(np.int64)
    return len(np.unique(key))


def rows_of_pass(cf, plane_pass):
    """(plane, MB-plane width, MB-plane height) per pass."""
    if plane_pass == 0:
        return [(0, 16, 16)]
    cw = 16 if cf == 3 else 8
    ch = 8 if cf == 1 else 16
    return [(1, cw, ch), (2, cw, ch)]


def luma2d_taps(P, mbs, stride, tw):
    """Luma taps of the 2-D lane layout (recon.hip Tap2, MP2VG_LUMA2D): lane (k, p, cx, m) loads
    OR + 1 rows of tw/4 + 1 dwords; instruction (direction, row i) spans every lane of the group.
    Instruction ids: group * 64 + 40 + direction * 8 + i."""
    n = len(mbs)
    mbw = int(P["mb_width"])
    x = mbs["x"].astype(np.int64)
    y = mbs["y"].astype(np.int64)
    fl = mbs["flags"].astype(np.int64)
    grp = (np.arange(n) // mbw) * ((mbw + 3) // 4) + (x // 4)
    inter = (fl & MB_INTRA) == 0
    use = [inter & (((fl & MB_FWD) != 0) | ((fl & MB_BWD) == 0)), inter & ((fl & MB_BWD) != 0)]
    field = (fl & MB_FIELD_MC) != 0
    orr, nc, nd = 64 // (4 * tw), 16 // tw, tw // 4 + 1
    st = stride[0]
    ids_l, lines_l, sec_l = [], [], []
    lanes = np.arange(16)  # per MB: (p, cx, m) of its 16 lanes
    p = lanes & 1
    cx = (lanes >> 1) & (nc - 1)
    m = lanes >> (1 + (nc.bit_length() - 1))
    for d in range(2):
        u = use[d]
        mvx = np.where(field[:, None], mbs["mv"][:, :, d, 0][:, p], mbs["mv"][:, 0, d, 0][:, None]).astype(np.int64)
        mvy = np.where(field[:, None], mbs["mv"][:, :, d, 1][:, p], mbs["mv"][:, 0, d, 1][:, None]).astype(np.int64)
        fs = (fl[:, None] >> (8 + 2 * p[None, :] + d)) & 1
        X = x[:, None] * 16 + cx[None, :] * tw + (mvx >> 1)
        Yf = y[:, None] * 16 + orr * (p[None, :] + 2 * m[None, :]) + (mvy >> 1)
        Yd = y[:, None] * 16 + fs + 2 * (orr * m[None, :] + (mvy >> 1))
        Y = np.where(field[:, None], Yd, Yf)
        step = np.where(field[:, None], 2, 1)
        sel = np.broadcast_to(u[:, None], Y.shape).ravel()
        gid = np.broadcast_to(grp[:, None], Y.shape).ravel()
        for i in range(orr + 1):
            a = ((Y + i * step) * st + (X & ~3)).ravel()
            ids = (gid * 64 + 40 + d * 8 + i)[sel]
            for addr in (a[sel], a[sel] + 4 * nd - 1):
                ids_l.append(ids)
                lines_l.append(addr >> 7)
                sec_l.append(addr >> 6)
    return np.concatenate(ids_l), np.concatenate(lines_l), np.concatenate(sec_l), grp


def picture_taps(P, mbs, stride, ph, plane_off, cf, layout, luma=True):
    """Arrays of (instruction id, line id, sector id) for every reference tap of one picture, and
    the group id of each instruction.  Instruction ids: group * 64 + kind."""
    n = len(mbs)
    mbw = int(P["mb_width"])
    x = mbs["x"].astype(np.int64)
    y = mbs["y"].astype(np.int64)
    fl = mbs["flags"].astype(np.int64)
    grp = (np.arange(n) // mbw) * ((mbw + 3) // 4) + (x // 4)
    inter = (fl & MB_INTRA) == 0
    use = [inter & (((fl & MB_FWD) != 0) | ((fl & MB_BWD) == 0)), inter & ((fl & MB_BWD) != 0)]
    field = (fl & MB_FIELD_MC) != 0
    out_ids, out_lines, out_sec = [], [], []
    kind = 0
    for ppass in ((0, 1) if luma else (1,)):
        for plane, pw, phm in rows_of_pass(cf, ppass):
            st = stride[plane]
            for d in range(2):
                u = use[d]
                if not u.any():
                    kind += 4
                    continue
                py = np.arange(phm)
                r = np.where(field[:, None], py[None, :] & 1, 0)
                mvx = np.where(r == 0, mbs["mv"][:, 0, d, 0][:, None], mbs["mv"][:, 1, d, 0][:, None]).astype(np.int64)
                mvy = np.where(r == 0, mbs["mv"][:, 0, d, 1][:, None], mbs["mv"][:, 1, d, 1][:, None]).astype(np.int64)
                if plane > 0:
                    if cf < 3:
                        mvx = mvx >> 1
                    if cf < 2:
                        mvy = mvy >> 1
                fs = (fl[:, None] >> (8 + 2 * r + d)) & 1
                X = x[:, None] * pw + (mvx >> 1)
                Yf = y[:, None] * phm + py[None, :] + (mvy >> 1)
                Yd = y[:, None] * phm + fs + 2 * ((py[None, :] >> 1) + (mvy >> 1))
                Y = np.where(field[:, None], Yd, Yf)
                step = np.where(field[:, None], 2, 1)
                hy = (mvy & 1) != 0
                edge = (py[None, :] + step) >= phm
                nbytes = 20 if pw == 16 else (12 if pw == 8 else 20)
                sel = np.broadcast_to(u[:, None], Y.shape)
                gid = np.broadcast_to(grp[:, None], Y.shape)
                if layout == "apron_h8" and plane == 0:
                    step = np.broadcast_to(step, Y.shape)
                    # half-row luma lanes (MB, r < 8, half h): instruction A = rows r, B = rows
                    # r + 8, E = the rows past 15 for the wrap lanes (r + step > 7) with vertical
                    # half-pel; one 12-B (b96) load per half row inside its apron tile row
                    for part, (rsel, msel) in enumerate((("A", None), ("B", None), ("E", None))):
                        for hh in range(2):
                            Xh = X + 8 * hh
                            if part == 0:
                                rows_, m_ = Y[:, :8], sel[:, :8]
                            elif part == 1:
                                rows_, m_ = Y[:, 8:], sel[:, 8:]
                            else:
                                rows_ = Y[:, 8:] + step[:, 8:]
                                wrap = (np.arange(8)[None, :] + step[:, 8:]) > 7
                                m_ = sel[:, 8:] & hy[:, 8:] & wrap
                            X0 = (Xh[:, :8] if part == 0 else Xh[:, 8:]) & ~3
                            XL = (X[:, :8] if part == 0 else X[:, 8:]) & ~3  # both halves in the left half's tile
                            t = (rows_ // 4) * -(-st // 16) + (XL // 16)
                            a = t * 128 + (rows_ % 4) * 32 + (X0 - 16 * (XL // 16))
                            m = m_.ravel()
                            ids = (np.broadcast_to(grp[:, None], rows_.shape).ravel() * 64 + kind * 4 + part)[m]
                            for addr in (a.ravel()[m], a.ravel()[m] + 11):
                                out_ids.append(ids)
                                out_lines.append(addr >> 7)
                                out_sec.append(addr >> 6)
                    kind += 1
                    continue
                for part, (rows, mask) in enumerate(((Y, sel), (Y + step, sel & hy & edge))):
                    X0 = X & ~3
                    if layout == "linear":
                        a = plane_off[plane] + rows * st + X0
                        spans = [(a, a + min(nbytes, 16) - 1, 0)] + ([(a + 16, a + nbytes - 1, 1)] if nbytes > 16 else [])
                    elif layout.startswith("apron"):  # one load per row inside a tile row with its apron
                        # apron: 4 rows x (16 + 16 apron) luma, 8 x (8 + 8) chroma (recon.hip tile_off);
                        # apron2: 2 rows x (48 + 16 apron) luma, 4 x (24 + 8) chroma (1.33x the bytes)
                        R_, OW = ((4, 16), (8, 8)) [plane > 0] if layout in ("apron", "apron_h8") else ((2, 48), (4, 24))[plane > 0]
                        t = (rows // R_) * -(-st // OW) + (X0 // OW)
                        a = (1 << 40) * plane + t * 128 + (rows % R_) * (128 // R_) + (X0 % OW)
                        spans = [(a, a + min(nbytes, 16) - 1, 0)] + ([(a + 16, a + nbytes - 1, 1)] if nbytes > 16 else [])
                    else:  # tile8x16: two loads per row (the row's left tile, then its right tile)
                        tw = 16 if plane == 0 else 16
                        th = 8
                        ta = (rows // th) * (st // tw) + (X0 // tw)
                        base = (1 << 40) * plane
                        a0 = base + ta * 128 + (rows % th) * tw
                        spans = [(a0, a0 + tw - 1, 0), (a0 + 128, a0 + 128 + tw - 1, 1)]
                    for lo, hi, sub in spans:
                        m = mask.ravel()
                        ids = (gid.ravel() * 64 + kind * 4 + part * 2 + sub)[m]
                        lo_, hi_ = lo.ravel()[m], hi.ravel()[m]
                        for addr in (lo_, hi_):
                            out_ids.append(ids)
                            out_lines.append(addr >> 7)
                            out_sec.append(addr >> 6)
                kind += 1
    return np.concatenate(out_ids), np.concatenate(out_lines), np.concatenate(out_sec), grp


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    config = args[0] if args else "c2"
    gops = int(args[1]) if len(args) > 1 else 8
    w, h, cf, gp, _ = bench.CONFIGS[config]
    es = R.generate_es(width=w, height=h, chroma_format=cf, n_gops=gops, seed=1729, **gp)
    parsed = R.Parsed(es, w, h, cf, threads=8)
    pw, ph, stride, slot_bytes = _lib.geometry(w, h, cf)
    plane_off = [0, stride[0] * ph[0], stride[0] * ph[0] + stride[1] * ph[1]]
    n = int(parsed.pics[0]["mb_width"]) * int(parsed.pics[0]["mb_height"])
    res = {}
    for layout in (sys.argv[sys.argv.index("--layouts") + 1].split(",") if "--layouts" in sys.argv else
                   ("linear", "apron", "apron2", "apron_h8", "tile8x16", "luma2d_tw8", "luma2d_tw4")):
        ta_l = ta_s = grp_l = groups = 0
        for p in range(parsed.npics):
            P = parsed.pics[p]
            if int(P["picture_coding_type"]) == 1:
                continue
            mbs = parsed.mbs[int(P["mb_first"]):int(P["mb_first"]) + n]
            if layout.startswith("luma2d"):
                ids, lines, secs, grp = picture_taps(P, mbs, stride, ph, plane_off, cf, "linear", luma=False)
                i2, l2, s2, _ = luma2d_taps(P, mbs, stride, int(layout[-1]))
                ids, lines, secs = np.concatenate([ids, i2]), np.concatenate([lines, l2]), np.concatenate([secs, s2])
            else:
                ids, lines, secs, grp = picture_taps(P, mbs, stride, ph, plane_off, cf, layout)
            ta_l += count_unique(ids, lines)
            ta_s += count_unique(ids, secs)
            grp_l += count_unique(ids // 64, lines)
            groups += int(grp.max()) + 1
        res[layout] = {"ta_line_lookups_per_group": ta_l / groups, "ta_sector_lookups_per_group": ta_s / groups,
                       "distinct_lines_per_group": grp_l / groups, "groups": groups}
    # row stores of P/B pictures (linear frame_c layout, 16-B luma / 8-B chroma rows): one line
    # per lane and instruction -- 64 per luma instruction, 64 per 4:2:0 chroma instruction
    npb = int(np.sum(parsed.pics["picture_coding_type"] != 1))
    scale = bench.DEFAULT_GOPS[config] / gops
    out = {"config": config, "gops_sampled": gops, "scale_to_step": scale, "pb_pictures": npb,
           "store_lines_per_group": 64 * (2 if cf == 1 else 3), "layouts": res}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""GOP sharding across ranks (one process per GPU).

Closed GOPs are independent (reference dependencies are only the two most recent anchors,
decoder.cpp:299-304, reset by each closed GOP's I picture), so a stream's GOPs are dealt
round-robin to ranks (GOP g -> rank g % world) and each rank decodes its share with no
data-path exchange.  The only collective is the frame gather after decode (digests or frames
to rank 0), done by the caller over RCCL (torch.distributed "nccl") or gloo in CPU tests.
"""
import numpy as np

from ._lib import MB_DTYPE, PIC_DTYPE


def gop_of_rank(gop_index, rank, world):
    return (np.asarray(gop_index) % world) == rank


def shard_batch(parsed, rank, world):
    """Sub-batch of `parsed` (records of a whole stream) holding the GOPs of `rank`.

    Returns (pics, mbs, coefs, picture_ids) with slots renumbered densely from 0 and MB /
    coefficient offsets rebased; picture_ids are the decode indices in the full stream.
    Raises ValueError if a picture of the shard references a picture of another shard (open
    GOP)."""
    keep = np.nonzero(gop_of_rank(parsed.gop, rank, world))[0]
    remap = {int(d): i for i, d in enumerate(keep)}
    nmb = int(parsed.pics[0]["mb_width"]) * int(parsed.pics[0]["mb_height"]) if len(parsed.pics) else 0
    pics = np.zeros(len(keep), PIC_DTYPE)
    mbs = np.zeros(len(keep) * nmb, MB_DTYPE)
    coef_chunks = []
    coef_base = 0
    for i, d in enumerate(keep):
        p = parsed.pics[d].copy()
        for f in ("fwd_slot", "bwd_slot"):
            ref = int(p[f])
            if ref < 0:
                continue
            used = _picture_uses(parsed, d, f)
            if ref not in remap:
                if used:
                    raise ValueError(f"picture {d} predicts from picture {ref} of another shard (open GOP)")
                p[f] = -1
            else:
                p[f] = remap[ref]
        p["dst_slot"] = i
        first = int(p["mb_first"])
        m = parsed.mbs[first:first + nmb].copy()
        c0 = int(m["coef_off"][0])
        c1 = int(m["coef_off"][-1]) + int(m["ncoef"][-1])
        m["coef_off"] = m["coef_off"] - c0 + coef_base
        coef_chunks.append(parsed.coefs[c0:c1])
        coef_base += c1 - c0
        p["mb_first"] = i * nmb
        pics[i] = p
        mbs[i * nmb:(i + 1) * nmb] = m
    coefs = np.concatenate(coef_chunks) if coef_chunks else np.zeros(0, np.uint32)
    return pics, mbs, coefs.astype(np.uint32), keep


def _picture_uses(parsed, d, field):
    first = int(parsed.pics[d]["mb_first"])
    nmb = int(parsed.pics[d]["mb_width"]) * int(parsed.pics[d]["mb_height"])
    fl = parsed.mbs["flags"][first:first + nmb].astype(np.int64)
    inter = (fl & 1) == 0
    if field == "fwd_slot":
        return bool(np.any(inter & (((fl & 2) != 0) | ((fl & 4) == 0))))
    return bool(np.any(inter & ((fl & 4) != 0)))

"""Collectives of the GOP-sharded decode: one process per GPU, no data-path
exchange; after decode, frames (or their digests) go to rank 0 in display order.

The reference's only cross-picture dependency is the two most recent anchors
(decoder.cpp:299-304), reset by each closed GOP's I picture, so GOP g is decoded on rank
g % world with nothing exchanged while decoding.  The one real exchange is the frame gather:

* gather_gops -- rank 0 receives every finished GOP's frames (packed Y|U|V, the reference
  sample's write_yuv layout, tiny_mp2v_dec.cpp:11-17) from the rank that decoded it, in display
  order, with one grouped send/recv (torch.distributed batch_isend_irecv; RCCL over xGMI with
  backend "nccl", gloo for the CPU tests) per round of `world` GOPs.  Rank 0's ingress
  (7 xGMI links) is below 8 GPUs' decode rate, so this is reported beside decode fps, never in it.
* gather_u64 -- per-frame device digests to every rank (the cheap parity gather).
* max_over_ranks -- the bench's max-over-ranks step time.

Works with any torch.distributed backend; `device` is the torch device of the tensors the
backend moves ("cuda:<local>" for nccl, "cpu" for gloo).
"""
import numpy as np


def max_over_ranks(value, dist, device="cpu"):
    import torch
    if dist is None:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_u64(arr, dist, device="cpu"):
    """all_gather of a uint64 array of any per-rank length -> list (one array per rank)."""
    import torch
    arr = np.ascontiguousarray(arr, np.uint64)
    if dist is None:
        return [arr]
    world = dist.get_world_size()
    n = torch.tensor([len(arr)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    pad = torch.zeros(max(sizes), dtype=torch.int64, device=device)
    pad[:len(arr)] = torch.from_numpy(arr.view(np.int64)).to(device)
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:k].cpu().numpy().view(np.uint64) for o, k in zip(outs, sizes)]


def gop_owner(ngops, world):
    """GOP g -> rank g % world (the sharding of tiny_mp2v_dec_amd.shard)."""
    return [g % world for g in range(ngops)]


def gather_gops(dist, gop_frames, gop_sizes, frame_bytes, device="cpu", dst=0):
    """Frame gather to `dst` in display order.

    gop_frames: {gop index: [frame tensors of this rank's GOP, display order]} -- uint8 tensors of
        frame_bytes on `device`, for the GOPs this rank owns (gop_owner).
    gop_sizes: frames per GOP, for every GOP of the stream (every rank knows the GOP structure).
    Returns, on dst, the list of all frames of the stream in display order (GOP by GOP); None on
    the other ranks.  One batch_isend_irecv per round of `world` consecutive GOPs, so every rank
    takes part in every grouped call and the sends of a round overlap on rank 0's links."""
    import torch
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    owner = gop_owner(len(gop_sizes), world)
    dev = torch.device(device)

    def on_backend_device(f):
        # a frame on another device than the backend moves (e.g. a cuda tensor under gloo, or a
        # host tensor under nccl) is copied over first: batch_isend_irecv needs one device
        return f if f.device == dev else f.to(dev)

    out = [] if rank == dst else None
    for r0 in range(0, len(gop_sizes), world):
        ops, recv = [], {}
        for g in range(r0, min(r0 + world, len(gop_sizes))):
            o = owner[g]
            if o == dst:
                if rank == dst:
                    recv[g] = [on_backend_device(f) for f in gop_frames[g]]
                continue
            if rank == o:
                if len(gop_frames[g]) != gop_sizes[g]:
                    raise ValueError(f"GOP {g}: {len(gop_frames[g])} frames, expected {gop_sizes[g]}")
                ops += [dist.P2POp(dist.isend, on_backend_device(f), dst) for f in gop_frames[g]]
            elif rank == dst:
                bufs = [torch.empty(frame_bytes, dtype=torch.uint8, device=device) for _ in range(gop_sizes[g])]
                ops += [dist.P2POp(dist.irecv, b, o) for b in bufs]
                recv[g] = bufs
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if rank == dst:
            for g in sorted(recv):
                out.extend(recv[g])
    return out

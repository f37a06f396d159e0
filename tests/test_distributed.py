"""CPU, world_size 2 over gloo: GOP sharding + the digest gather that bench.py does over RCCL.

Each rank takes GOPs g % world == rank of one stream, reconstructs its shard (here with the
oracle, as the CPU stand-in for the HIP kernel), computes per-frame digests, and all_gathers
them to every rank; the union must equal the single-process decode of the whole stream.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, es, q):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    import torch
    from helpers import oracle_frames
    from tiny_mp2v_dec_amd.records import Parsed, planes_digest
    from tiny_mp2v_dec_amd.shard import shard_batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parsed = Parsed(es, 176, 144, 1)
    pics, mbs, coefs, ids = shard_batch(parsed, rank, world)

    class P:
        pass

    sp = P()
    sp.width, sp.height, sp.chroma_format = 176, 144, 1
    sp.pics, sp.mbs, sp.coefs, sp.npics = pics, mbs, coefs, len(pics)
    frames = oracle_frames(sp)
    local = torch.tensor([[int(i), planes_digest(f) - (1 << 63)] for i, f in zip(ids, frames)], dtype=torch.int64)
    n = torch.tensor([len(local)])
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = torch.full((mx, 2), -1, dtype=torch.int64)
    pad[:len(local)] = local
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    if rank == 0:
        got = {}
        for o in outs:
            for i, d in o.tolist():
                if i >= 0:
                    got[i] = d + (1 << 63)
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gop_shard_gather_equals_single_process(world):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    from helpers import oracle_frames
    from tiny_mp2v_dec_amd.records import Parsed, generate_es, planes_digest

    es = generate_es(width=176, height=144, chroma_format=1, n_gops=3, gop_n=6, gop_m=3, seed=77)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, es, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = Parsed(es, 176, 144, 1)
    exp = {i: planes_digest(f) for i, f in enumerate(oracle_frames(full))}
    assert got == exp


def test_shard_rejects_open_gop_cross_reference():
    import sys
    sys.path[:0] = [REPO]
    from tiny_mp2v_dec_amd.records import Parsed, generate_es
    from tiny_mp2v_dec_amd.shard import shard_batch
    es = generate_es(width=176, height=144, chroma_format=1, n_gops=2, gop_n=6, gop_m=3, seed=5)
    p = Parsed(es, 176, 144, 1)
    # make picture 7's forward reference point into GOP 0 and mark an MB as using it
    p.gop[:] = np.arange(p.npics) // 6
    d = 7
    if p.pics[d]["picture_coding_type"] == 1:
        d = 8
    p.pics[d]["fwd_slot"] = 0
    first = int(p.pics[d]["mb_first"])
    p.mbs["flags"][first] = 2
    with pytest.raises(ValueError):
        shard_batch(p, 1, 2)


def _gather_worker(rank, world, port, es, q):
    """GOP-sharded decode (oracle as the CPU stand-in for the kernel) + the collectives bench.py
    runs: max-over-ranks time, the digest all_gather and the rank-0 frame gather in display order."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    import torch
    from helpers import oracle_frames
    from tiny_mp2v_dec_amd import gather as G
    from tiny_mp2v_dec_amd.records import Parsed, frame_yuv_bytes
    from tiny_mp2v_dec_amd.shard import shard_batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parsed = Parsed(es, 176, 144, 1)
    pics, mbs, coefs, ids = shard_batch(parsed, rank, world)

    class P:
        pass

    sp = P()
    sp.width, sp.height, sp.chroma_format = 176, 144, 1
    sp.pics, sp.mbs, sp.coefs, sp.npics = pics, mbs, coefs, len(pics)
    frames = dict(zip((int(i) for i in ids), oracle_frames(sp)))  # full-stream decode index -> planes
    ngops = int(parsed.gop.max()) + 1
    sizes = [int(np.sum(parsed.gop == g)) for g in range(ngops)]
    mine = {}
    for g in range(ngops):
        if g % world == rank:
            disp = [int(d) for d in parsed.display if parsed.gop[d] == g]
            mine[g] = [torch.from_numpy(np.frombuffer(frame_yuv_bytes(frames[d]), np.uint8).copy()) for d in disp]
    fb = 176 * 144 * 3 // 2
    got = G.gather_gops(dist, mine, sizes, fb)
    mx = G.max_over_ranks(float(rank + 1), dist)
    u = G.gather_u64(np.arange(rank + 2, dtype=np.uint64) + np.uint64(1 << 63), dist)
    if rank == 0:
        q.put(([bytes(t.numpy()) for t in got], mx, [x.tolist() for x in u]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank0_frame_gather_display_order(world):
    """gather.gather_gops over gloo: rank 0 ends with every frame of the stream in display order,
    byte-identical to a single-process decode written in the reference's write_yuv layout."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    from helpers import oracle_frames
    from tiny_mp2v_dec_amd.records import Parsed, frame_yuv_bytes, generate_es

    es = generate_es(width=176, height=144, chroma_format=1, n_gops=4, gop_n=6, gop_m=3, seed=78)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, es, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, mx, u = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = Parsed(es, 176, 144, 1)
    fr = oracle_frames(full)
    assert got == [frame_yuv_bytes(fr[d]) for d in full.display]
    assert mx == float(world)
    assert u == [[(1 << 63) + k for k in range(r + 2)] for r in range(world)]


def _bench_phase_worker(rank, world, port, q, bad_rank):
    """bench.py's distributed phases -- init_distributed (the torch.distributed.run environment),
    parity_over_ranks and frame_gather -- exactly as bench.py calls them at N > 1, with the oracle
    standing in for the kernel: each rank decodes its own stream (seed 1729 + rank)."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch
    import bench
    from helpers import oracle_frames
    from tiny_mp2v_dec_amd.records import Parsed, frame_yuv_bytes, generate_es, planes_digest

    r, w, d, coll_dev, device = bench.init_distributed("gloo")
    assert (r, w, coll_dev, device) == (rank, world, "cpu", 0) and d is not None
    es = generate_es(width=176, height=144, chroma_format=1, n_gops=3, gop_n=6, gop_m=3, seed=1729 + rank)
    parsed = Parsed(es, 176, 144, 1)
    frames = oracle_frames(parsed)
    dig = np.array([planes_digest(f) for f in frames], np.uint64)
    exp = dig.copy()
    if rank == bad_rank:
        exp[1] ^= np.uint64(1)
    parity, gathered = bench.parity_over_ranks(dig, exp, d, coll_dev)

    def copy_frame(i, t, on_dev):
        assert not on_dev and t.device == torch.device(coll_dev)
        t.copy_(torch.from_numpy(np.frombuffer(frame_yuv_bytes(frames[i]), np.uint8).copy()))

    pw, ph = [176, 88, 88], [144, 72, 72]
    res = bench.frame_gather(d, coll_dev, parsed, 176 * 144 * 3 // 2, copy_frame, pw, ph, gathered, 2)
    if rank == 0:
        q.put((parity, res, [len(g) for g in gathered]))
    d.barrier()
    d.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [-1, 1])
def test_bench_distributed_phases_gloo(bad_rank):
    """bench.py's N > 1 code (the functions the nccl run calls, here over gloo on CPU tensors):
    every rank's digests reach rank 0, parity is bit-exact -- or names the rank whose digests
    differ -- and the rank-0 frame gather of two GOPs per rank verifies in display order."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_phase_worker, args=(r, world, port, q, bad_rank)) for r in range(world)]
    for p in procs:
        p.start()
    parity, res, lens = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert lens == [18, 18]
    if bad_rank < 0:
        assert parity["status"] == "bit-exact" and parity["frames_checked"] == 36
    else:
        assert parity == {"status": "MISMATCH", "ranks_mismatching": [bad_rank]}
    assert res["verified"] and res["frames"] == 2 * 2 * 6


def test_gather_gops_sends_on_the_backend_device():
    """Every frame handed to the grouped send is on the backend's device (gather_gops copies a
    frame from another device first: a cuda frame under gloo, a host frame under nccl); here with
    a stand-in distributed module that records what it is asked to send."""
    import sys
    sys.path[:0] = [REPO]
    import torch
    from tiny_mp2v_dec_amd import gather as G

    sent = []

    class FakeDist:
        isend, irecv = "isend", "irecv"

        @staticmethod
        def get_rank():
            return 1

        @staticmethod
        def get_world_size():
            return 2

        class P2POp:
            def __init__(self, op, t, peer):
                sent.append((op, t, peer))

        @staticmethod
        def batch_isend_irecv(ops):
            return []

    frames = {1: [torch.zeros(8, dtype=torch.uint8), torch.ones(8, dtype=torch.uint8)]}
    G.gather_gops(FakeDist, frames, [3, 2], 8, device="cpu")
    assert [(op, peer) for op, _, peer in sent] == [("isend", 0), ("isend", 0)]
    assert all(t.device == torch.device("cpu") for _, t, _ in sent)


@pytest.mark.parametrize("config,ranks,gops", [("c2", 8, None), ("c4", 8, None), ("c4", 8, 1)])
def test_reference_digests_for_every_rank_of_the_scaling_run(config, ranks, gops):
    """The driver's 1/2/4/8-GPU bench runs give rank r the stream of seed 1729 + r: the compiled
    reference's per-frame digests exist for every rank, so parity is checked on all of them (and
    for the one-GOP c4 rehearsal of the 8-rank command, tests/test_bench_multirank.py)."""
    import sys
    sys.path[:0] = [REPO]
    import bench
    import numpy as np
    with np.load(os.path.join(REPO, "tests", "golden", "bench_digests.npz")) as d:
        # the entries were computed with the formula bench.py's device digests use
        assert int(d["digest_format"][0]) == bench.DIGEST_FORMAT
    gops = gops or bench.DEFAULT_GOPS[config]
    for r in range(ranks):
        exp = bench.expected_digests(config, gops, 1729 + r)
        assert exp is not None and len(exp) == 12 * gops, (config, r)


def test_plain_bench_gpus_2_spawns_two_ranks():
    """`python bench.py --gpus 2` (no launcher, the form of the driver's BENCH command) starts two
    ranks itself -- one torch.distributed.run child, before any torch import or GPU call in the
    parent -- and they form a world-2 group (gloo here; nccl on a GPU node)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--probe-launch"], capture_output=True, text=True, timeout=240, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks"] == [0, 1] and lines[0]["max_rank"] == 1.0


def test_plain_bench_gpus_8_c4_spawns_eight_ranks():
    """The c4 scaling command's launch, `python bench.py --gpus 8 --config c4` with no launcher:
    eight ranks over gloo form one world, each knows its rank, and max-over-ranks sees all of them."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "8", "--config", "c4", "--gops", "1",
                        "--backend", "gloo", "--probe-launch"], capture_output=True, text=True, timeout=300, cwd=repo,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    assert lines[0]["n_gpus"] == 8 and lines[0]["ranks"] == list(range(8)) and lines[0]["max_rank"] == 7.0


def test_bench_refuses_a_world_that_does_not_match_gpus():
    """Under a launcher, --gpus must equal the launched world (a --gpus 8 line can never come
    from one rank)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port_here()))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--probe-launch"], capture_output=True, text=True, timeout=240, cwd=repo, env=env)
    assert r.returncode != 0 and "--gpus 2 but the launcher started 1 rank" in r.stderr


def _free_port_here():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p

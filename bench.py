"""Benchmark: MPEG-2 macroblock reconstruct on MI355X (BASELINE.json metric / configs[1]).

A "step" = one pass of the hot path over one batch: the dequant + IDCT + MC + add/clip of every
picture of G closed GOPs (1080p 4:2:0, N=12, M=3 -> 12*G frames) whose pre-parsed macroblock
records are already resident in HBM.  Each rank (one per GPU) decodes its own independent GOP
stream (seed 1729 + rank): weak scaling, no data-path collective; RCCL only gathers per-frame
digests to rank 0 after the timed region (the trivial frame gather).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--gops G] [--config c1|c2|c3|c4|c5]

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks_if_needed(argv):
    """`python bench.py --gpus N` with N > 1 outside a torch.distributed launcher: run the N ranks
    (one process per GPU) as ONE child, `python -m torch.distributed.run --nproc-per-node N`, on
    127.0.0.1, forward its output and exit with its status.  This process never imports torch
    and never touches a GPU (an exec from a GPU-initialised process is forbidden on this pool).
    Under a launcher (WORLD_SIZE set) nothing happens here and main() checks world == --gpus."""
    if "WORLD_SIZE" in os.environ:
        return
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args(argv)
    if known.gpus <= 1:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    sys.stdout.flush()
    sys.exit(subprocess.run(cmd).returncode)


if __name__ == "__main__":
    spawn_ranks_if_needed(sys.argv[1:])

from tiny_mp2v_dec_amd import build as _build  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

BASELINE_METRIC = "decoded frames/sec + GB/s vs HBM roofline, 1080p 4:2:0 @1/2/4/8 GPU; bit-exact YUV"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

CONFIGS = {
    # name: (width, height, chroma_format, generator params, description)
    # c1 = BASELINE configs[0]: the reference's own CPU-runnable case (I-only, normal intra bitrate:
    # 0-12 AC coefficients per block), timed on the reference single-threaded beside the HIP path
    "c1": (1920, 1088, 1, dict(gop_n=1, gop_m=1, mix=1), "1080p 4:2:0 progressive I-only (120 frames)"),
    "c2": (1920, 1088, 1, dict(gop_n=12, gop_m=3, leading_b=1), "1080p 4:2:0 IPB GOP=12 (N=12, M=3, closed)"),
    "c3": (1920, 1088, 2, dict(gop_n=12, gop_m=3, leading_b=1), "1080p 4:2:2 IPB GOP=12 (N=12, M=3, closed)"),
    "c4": (3840, 2160, 1, dict(gop_n=12, gop_m=3, leading_b=1), "4K 4:2:0 IPB GOP=12 (N=12, M=3, closed)"),
    "c5": (1920, 1088, 3, dict(gop_n=1, gop_m=1, mix=1, intra_coefs_min=20, intra_coefs_max=40),
           "1080p 4:4:4 I-only high bitrate (20-40 AC coefficients per block)"),
}


# GOPs per GPU per step (c1, c5: I-only, one picture per "GOP").  The IPB configs keep ~10 GB of
# frames resident per step (c2: 3,072 frames = 9.6 GB; c3: 3,072 frames = 12.8 GB; c4: 4K, 768 frames =
# 9.5 GB): level launches 4x longer than at the earlier 64 / 64 / 16 GOPs amortise their ramps and
# tails (same box: c2 337.5k vs 328.3k, c3 256.0k vs 234.6k, c4 89.0k vs 83.1k frames/s;
# profiles/r3/README.md)
DEFAULT_GOPS = {"c1": 120, "c2": 256, "c3": 256, "c4": 64, "c5": 64}


def algorithmic_bytes(parsed):
    """B_out + B_ref + B_rec for the batch.
    B_out = visible plane bytes per frame; B_ref = 384/512/768 B per predicted MB per direction;
    B_rec = 32 B per MB record + 4 B per coefficient word (intra DC counted as one)."""
    cf = parsed.chroma_format
    w, h = parsed.width, parsed.height
    cw = w if cf == 3 else w // 2
    ch = h if cf != 1 else h // 2
    frame = w * h + 2 * cw * ch
    mb_bytes = {1: 384, 2: 512, 3: 768}[cf]
    fl = parsed.mbs["flags"].astype(np.int64)
    inter = (fl & 1) == 0
    fwd = ((fl & 2) != 0) | (inter & ((fl & 4) == 0))
    bwd = (fl & 4) != 0
    dirs = int(np.sum(inter * (fwd.astype(np.int64) + bwd.astype(np.int64))))
    b_out = frame * parsed.npics
    b_ref = dirs * mb_bytes
    b_rec = 32 * len(parsed.mbs) + 4 * len(parsed.coefs)
    return b_out + b_ref + b_rec, dict(out=b_out, ref=b_ref, rec=b_rec)


def per_picture_bytes(parsed):
    """algorithmic_bytes split by picture (decode order): frame bytes + its MBs' reference bytes +
    its records and coefficient words.  Summed per kernel launch for the per-kernel roofline."""
    cf = parsed.chroma_format
    w, h = parsed.width, parsed.height
    cw = w if cf == 3 else w // 2
    ch = h if cf != 1 else h // 2
    frame = w * h + 2 * cw * ch
    mb_bytes = {1: 384, 2: 512, 3: 768}[cf]
    n = int(parsed.pics[0]["mb_width"]) * int(parsed.pics[0]["mb_height"])
    fl = parsed.mbs["flags"].astype(np.int64).reshape(parsed.npics, n)
    inter = (fl & 1) == 0
    dirs = inter * ((((fl & 2) != 0) | (inter & ((fl & 4) == 0))).astype(np.int64) + ((fl & 4) != 0))
    ncoef = parsed.mbs["ncoef"].astype(np.int64).reshape(parsed.npics, n)
    return frame + mb_bytes * dirs.sum(1) + 32 * n + 4 * ncoef.sum(1)


# records.planes_digest's formula (2: mix64(mix64((row << 32) | x) ^ d), round 4); the golden
# digest file records the format its entries were computed with
DIGEST_FORMAT = 2


def expected_digests(config, gops, seed):
    """Per-slot (decode order) frame digests of this bench workload from the compiled reference
    (tests/golden/bench_digests.npz, written by tests/golden/make_bench_digests.py), or None."""
    path = os.path.join(REPO, "tests", "golden", "bench_digests.npz")
    if not os.path.exists(path):
        return None
    with np.load(path) as d:
        fmt = int(d["digest_format"][0]) if "digest_format" in d.files else 1
        if fmt != DIGEST_FORMAT:
            raise SystemExit(f"{path}: digest format {fmt}, this build computes format {DIGEST_FORMAT} "
                             "(tests/golden/make_bench_digests.py)")
        key = f"{config}_g{gops}_s{seed}"
        return d[key].copy() if key in d else None


def cpu_baseline(es, width, height, cf, frames):
    """The REAL reference (oracle/_ref/ref_decode, x86 SSE2, its own multithreaded path) on the
    same stream, timed on this host.  Falls back to the oracle C port when the prebuilt
    reference binary is absent."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 2)
    threads = max(1, min(share, os.cpu_count() or share) - 2)
    ref = os.path.join(REPO, "oracle", "_ref", "ref_decode")
    if os.path.exists(ref):
        with tempfile.NamedTemporaryFile(suffix=".m2v", delete=False) as f:
            f.write(es)
            path = f.name
        try:
            res = {}
            for t in (1, threads):
                r = subprocess.run([ref, path, str(width), str(height), str(cf), str(t), "-", "2"],
                                   capture_output=True, text=True, timeout=600)
                if r.returncode != 0:
                    raise RuntimeError(r.stderr[-300:])
                res[t] = json.loads(r.stdout.strip().splitlines()[-1])
        finally:
            os.unlink(path)
        mt = res[threads]
        return {"value": round(mt["frames"] / (mt["ms"] / 1000.0), 2), "unit": "frames/s", "cores": threads,
                "kind": "reference",
                "sample": f"whole bench stream ({mt['frames']} frames), reference decode() incl. VLC parse, "
                          f"best of 2; 1-thread: {res[1]['frames'] / (res[1]['ms'] / 1000.0):.1f} frames/s",
                "value_1thread": round(res[1]["frames"] / (res[1]["ms"] / 1000.0), 2)}
    # oracle port (records -> pixels, single thread)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle
    parsed = R.Parsed(es, width, height, cf)
    t0 = time.perf_counter()
    _oracle.reconstruct(width, height, cf, parsed.pics, parsed.mbs, parsed.coefs, parsed.npics)
    dt = time.perf_counter() - t0
    return {"value": round(parsed.npics / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"oracle C restatement over the bench records ({parsed.npics} frames), no parse"}


def profiled_traffic(config, gops):
    """HBM bytes per step of this exact workload from the committed rocprofv3 PMC summary
    (profiles/traffic_<config>_g<gops>.json, written by tools/prof_summary.py --json from
    tools/profile.sh's separate FETCH_SIZE / WRITE_SIZE passes of this bench command), or None."""
    path = os.path.join(REPO, "profiles", f"traffic_{config}_g{gops}.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    d["source"] = f"profiles/{os.path.basename(path)} ({d.get('tag')})"
    return d


def init_distributed(backend):
    """One process per GPU (torch.distributed.run env).  nccl (= RCCL on ROCm): the rank's GPU is
    set first and the process group is bound to it (device_id: eager communicator init), and the
    collectives move cuda tensors; gloo: CPU tensors (several ranks may share one GPU).
    Returns (rank, world, dist or None, collective device, local GPU index)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    ndev = max(1, torch.cuda.device_count())  # does not initialise the GPU
    device = local_rank % ndev
    dist, coll_dev = None, "cpu"
    # under a launcher the process group is formed even at world 1 (a one-rank RCCL run executes
    # every collective of the N-GPU path on one MI355X: tests/test_bench_multirank.py)
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as tdist
        if backend == "nccl":
            torch.cuda.set_device(device)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", device))
            coll_dev = f"cuda:{device}"
        else:
            tdist.init_process_group("gloo")
        dist = tdist
    return rank, world, dist, coll_dev, device


def parity_over_ranks(dig, exp, dist, coll_dev):
    """Every rank's frame digests vs the compiled reference's (exp, or None when the workload has
    none), gathered to all ranks.  Returns (parity record, per-rank digest arrays)."""
    from tiny_mp2v_dec_amd import gather as G
    my_status = 2 if exp is None else (1 if np.array_equal(dig, exp) else 0)  # 2 unchecked, 1 ok, 0 bad
    gathered = G.gather_u64(dig, dist, coll_dev)
    statuses = [int(x[0]) for x in G.gather_u64(np.array([my_status], np.uint64), dist, coll_dev)]
    if any(s == 0 for s in statuses):
        parity = {"status": "MISMATCH", "ranks_mismatching": [r for r, s in enumerate(statuses) if s == 0]}
    elif all(s == 1 for s in statuses):
        parity = {"status": "bit-exact", "frames_checked": int(sum(len(g) for g in gathered)),
                  "against": "tests/golden/bench_digests.npz: per-frame digests of the compiled reference "
                             "decoder (1 thread) on each rank's stream"}
    else:
        parity = {"status": "unchecked", "why": "no reference digests for this workload/seed in "
                                                "tests/golden/bench_digests.npz"}
    return parity, gathered


def frame_gather(dist, coll_dev, parsed, fb, copy_frame, pw, ph, gathered, gather_gops):
    """The rank-0 frame gather of the first `gather_gops` GOPs of every rank (GOP g of the virtual
    stream = GOP g // world of rank g % world), display order, timed with max over ranks; rank 0
    spot-checks the first and last frame of two GOPs per rank against that rank's digests.
    copy_frame(decode index, uint8 tensor on coll_dev, on_device) packs a decoded frame."""
    import torch
    from tiny_mp2v_dec_amd import gather as G
    rank, world = dist.get_rank(), dist.get_world_size()
    ng = min(gather_gops, int(parsed.gop.max()) + 1)
    on_dev = coll_dev != "cpu"
    gop_sizes, gop_frames = [], {}
    for g in range(ng * world):
        local = [int(d) for d in parsed.display if parsed.gop[d] == g // world]
        gop_sizes.append(len(local))
        if g % world == rank:
            fr = []
            for d in local:
                t = torch.empty(fb, dtype=torch.uint8, device=coll_dev)
                copy_frame(d, t, on_dev)
                fr.append(t)
            gop_frames[g] = fr
    if on_dev:
        torch.cuda.synchronize()
    dist.barrier()
    tg = time.perf_counter()
    got = G.gather_gops(dist, gop_frames, gop_sizes, fb, device=coll_dev)
    if on_dev:
        torch.cuda.synchronize()
    tg = G.max_over_ranks(time.perf_counter() - tg, dist, coll_dev)
    res = None
    if rank == 0:
        # every rank's stream has the same GOP structure, so rank 0's own display order and GOP
        # index map a gathered position to the sender's decode index
        starts = np.concatenate([[0], np.cumsum(gop_sizes)])
        ok = True
        for r in range(min(world, ng * world)):
            for g in (r, r + world * (ng - 1)):
                local = [int(d) for d in parsed.display if parsed.gop[d] == g // world]
                for k in (0, len(local) - 1):
                    buf = got[int(starts[g]) + k].cpu().numpy()
                    planes, o = [], 0
                    for i in range(3):
                        planes.append(buf[o:o + pw[i] * ph[i]].reshape(ph[i], pw[i]))
                        o += pw[i] * ph[i]
                    ok &= R.planes_digest(planes) == int(gathered[r][local[k]])
        res = {"frames": len(got), "bytes": int(len(got) * fb), "ms": round(tg * 1e3, 3),
               "GBps_into_rank0": round(len(got) * fb / tg / 1e9, 2), "verified": bool(ok),
               "sample": f"first {ng} GOPs of every rank, frame by frame in display order"}
    del gop_frames, got
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gops", type=int, default=None, help="GOPs per GPU (default: DEFAULT_GOPS[config])")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (gloo: CPU collectives; lets several ranks "
                         "share one GPU to rehearse the multi-GPU path)")
    ap.add_argument("--gather-gops", type=int, default=8,
                    help="GOPs per rank in the rank-0 frame gather measured after the timed region")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the drop-in end-to-end measurement")
    ap.add_argument("--probe-launch", action="store_true",
                    help="form the process group, check world == --gpus with one all_reduce, print one JSON "
                         "line and exit before any GPU work (CPU test of the N-rank launch)")
    args = ap.parse_args()

    rank, world, dist, coll_dev, device = init_distributed(args.backend)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.probe_launch:
        from tiny_mp2v_dec_amd import gather as G
        ranks = G.gather_u64(np.array([rank], np.uint64), dist, coll_dev)
        mx = G.max_over_ranks(rank, dist, coll_dev)
        if rank == 0:
            print(json.dumps({"probe": "launch", "n_gpus": world, "backend": args.backend if dist else None,
                              "ranks": [int(r[0]) for r in ranks], "max_rank": mx}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    import torch

    if rank == 0:
        _build.build()
    if dist is not None:
        dist.barrier()

    from tiny_mp2v_dec_amd import gather as G

    width, height, cf, gparams, desc = CONFIGS[args.config]
    # c5 is I-only: one picture per "GOP", so --gops is its frame count (~60 frames; at
    # 768 frames its elementary stream would pass the 2 GB `int len` of the reference decode() API)
    gops = args.gops or DEFAULT_GOPS[args.config]
    seed = 1729 + rank
    es = R.generate_es(width=width, height=height, chroma_format=cf, n_gops=gops, seed=seed, **gparams)
    parsed = R.Parsed(es, width, height, cf, threads=min(8, os.cpu_count() or 1))
    alg_bytes, parts = algorithmic_bytes(parsed)
    ctx = R.DeviceContext(width, height, cf, slots=parsed.npics, device=device)
    ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)
    # the one-stream context of the per-kernel lines (used after the timed region); with
    # MP2VG_BENCH_CTX1_EARLY=1 (measurements) it takes its pool now, before ctx's first batch
    ctx1 = None
    if os.environ.get("MP2VG_BENCH_CTX1_EARLY") == "1":
        ctx1 = R.DeviceContext(width, height, cf, slots=parsed.npics, device=device, one_stream=True)
        ctx1.upload(parsed.pics, parsed.mbs, parsed.coefs)

    for _ in range(args.warmup):
        ctx.decode()
    ctx.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    ctx.synchronize()
    # steps are enqueued back to back (no host sync between them); each step's HIP events (around
    # each launch, and first launch start -> last launch end) are read after the timed region
    timed = min(args.steps, 64)  # mp2vg_batch_times keeps the last 64 batches
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.decode()
    ctx.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms, batch_ms = [], []
    for back in range(timed - 1, -1, -1):
        b, l = ctx.batch_times(back)
        batch_ms.append(b)
        kernel_ms.append(l)
    # device span of the timed steps: first batch start -> last batch end (consecutive batches
    # overlap picture set by picture set, runtime.cpp mp2vg_batch_decode)
    device_span_ms = ctx.batches_span(timed - 1, 0)
    # the runtime's pool placement calibration at the context's first (warm-up) batch
    place_ms, place_kept = ctx.placement()
    elapsed = G.max_over_ranks(elapsed, dist, coll_dev)

    # ---- parity of the timed batch: device digest of every frame vs the compiled reference's ----
    dig = ctx.digests(np.arange(parsed.npics))
    exp = expected_digests(args.config, gops, seed)
    parity, gathered = parity_over_ranks(dig, exp, dist, coll_dev)

    # ---- per-kernel roofline: the same batch on a one-stream context, so launches never overlap ----
    of_pic, modes = R.plan_batch(width, height, cf, parsed.npics, parsed.pics, parsed.mbs, parsed.coefs,
                                 one_stream=True)
    pic_bytes = per_picture_bytes(parsed)
    launch_bytes = np.bincount(of_pic, weights=pic_bytes, minlength=len(modes))
    if ctx1 is None:
        ctx1 = R.DeviceContext(width, height, cf, slots=parsed.npics, device=device, one_stream=True)
        ctx1.upload(parsed.pics, parsed.mbs, parsed.coefs)
    k1 = 5
    for _ in range(k1 + 1):
        ctx1.decode()
    ctx1.synchronize()
    l1 = np.array([ctx1.batch_times(back)[1] for back in range(k1)])  # (k1, launches)
    span1 = float(np.mean([ctx1.batch_times(back)[0] for back in range(k1)]))
    if exp is not None and not np.array_equal(ctx1.digests(np.arange(parsed.npics)), exp):
        parity = {"status": "MISMATCH", "ranks_mismatching": [rank], "context": "one-stream"}
    ctx1.close()
    per_kernel = {}
    for m in sorted(set(modes.tolist())):
        sel = modes == m
        ms = float(l1[:, sel].mean(axis=0).sum())
        nbytes = float(launch_bytes[sel].sum())
        name = f"recon_kernel<{cf}, {m}, 0>"
        per_kernel[name] = {"mode": ["I", "P / one-direction B", "B", "P+B", "I, tiles converted after"][m], "launches_per_step": int(sel.sum()),
                            "avg_launch_ms": round(ms / int(sel.sum()), 4),
                            "algorithmic_bytes_per_launch": int(nbytes / int(sel.sum())),
                            "achieved_GBps": round(nbytes / (ms / 1e3) / 1e9, 1),
                            "frac": round(nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                            "share_of_step": round(ms / float(l1.sum(axis=1).mean()), 3)}
    dominant = max(per_kernel, key=lambda k: per_kernel[k]["share_of_step"])

    # ---- rank-0 frame gather (grouped send/recv per round of GOPs, display order), timed apart ----
    gather_res = None
    if dist is not None:
        gather_res = frame_gather(dist, coll_dev, parsed, ctx.frame_bytes(),
                                  lambda d, t, on_dev: ctx.copy_packed(d, t.data_ptr(), on_dev),
                                  ctx.pw, ctx.ph, gathered, args.gather_gops)

    # this box's shader clock under a VALU load on every SIMD (s_memtime against the 100-MHz
    # s_memrealtime), measured after the timed region: the per-box record behind the box-to-box
    # spread of the step (profiles/r6/README.md)
    import ctypes
    from tiny_mp2v_dec_amd._lib import lib as _native
    ghz = ctypes.c_double(0.0)
    clock_ghz = round(ghz.value, 3) if _native().mp2vg_clock_probe(device, ctypes.byref(ghz)) == 0 else None

    traffic = profiled_traffic(args.config, gops)
    frames_total = parsed.npics * world * args.steps
    ms_per_step = elapsed * 1000.0 / args.steps
    per_launch = [x for step in kernel_ms for x in step]
    # the kernel time of a step: the device span of the timed steps (HIP events on the launch
    # streams, first batch start -> last batch end, gaps between launches included) / steps
    kernel_step_ms = device_span_ms / timed
    achieved = alg_bytes / (kernel_step_ms / 1000.0) / 1e9
    result = {
        "metric": BASELINE_METRIC,
        "value": round(frames_total / elapsed, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"{desc}, pre-parsed MB records resident in HBM, {gops} GOPs per GPU",
                   "width": width, "height": height, "chroma_format": {1: "4:2:0", 2: "4:2:2", 3: "4:4:4"}[cf],
                   "frames_per_gpu_per_step": parsed.npics, "global_batch_frames": parsed.npics * world,
                   "parallelism": f"gop-shard x{world}", "backend": args.backend if dist is not None else None},
        "parity": parity,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic["traffic_bytes_per_step"] if traffic else None,
                     "traffic_unit": "bytes/step (HBM, PMC)", "traffic_source": traffic["source"] if traffic else None,
                     "traffic_fetch_raw": traffic.get("fetch_raw_bytes_per_step") if traffic else None,
                     "traffic_write": traffic.get("write_bytes_per_step") if traffic else None,
                     "l2_requests_per_step": traffic.get("l2_requests_per_step") if traffic else None,
                     "l2_hit_rate": traffic.get("l2_hit_rate") if traffic else None,
                     # on-chip bound: L1->L2 request bytes over the algorithmic bytes, at 64 B per
                     # request (the sector a 20-B tap row or a 64-B store quad needs) and at the
                     # 128-B line a read request fills (tools/fetch_calib.hip): lower / upper bound
                     "l1l2_amplification": (round(traffic["l2_requests_per_step"] * 64 / alg_bytes, 3)
                                            if traffic and traffic.get("l2_requests_per_step") else None),
                     "l1l2_amplification_128B": (round(traffic["l2_requests_per_step"] * 128 / alg_bytes, 3)
                                                 if traffic and traffic.get("l2_requests_per_step") else None),
                     "kernel": "mp2vg::recon_kernel", "launches_per_step": len(kernel_ms[0]),
                     "avg_launch_ms": round(float(np.mean(per_launch)), 4),
                     "algorithmic_bytes_per_step": int(alg_bytes), "bytes_breakdown": parts,
                     "kernel_ms_per_step": round(kernel_step_ms, 4),
                     "batch_span_ms": round(float(np.mean(batch_ms)), 4),
                     "sum_launch_ms_per_step": round(float(np.mean([sum(s) for s in kernel_ms])), 4),
                     "dominant_kernel": dominant, "one_stream_span_ms": round(span1, 4),
                     "per_kernel": per_kernel},
        "box": {"shader_clock_ghz_valu_load": clock_ghz, "host_cpus_visible": os.cpu_count()},
        "pool_placement": {"candidate_batch_ms": place_ms, "kept": place_kept,
                           "note": "runtime.cpp calibrate_placement, at the first warm-up batch: the batch "
                                   "decoded on the pool and on copies in fresh blocks (round 0 of each, then "
                                   "round 1), the fastest pool kept; outside the timed region"},
        "frame_digest_of_digests": int(np.bitwise_xor.reduce(np.concatenate(gathered))),
        "provenance": _build.provenance(),
    }
    if gather_res is not None:
        result["frame_gather"] = gather_res
    ctx.close()
    if rank == 0 and world == 1 and dist is None and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(es, width, height, cf, parsed.npics)
    if rank == 0 and world == 1 and dist is None and not args.no_e2e:
        result["e2e_dropin"] = e2e_dropin(es, width, height, cf, parsed.npics, device,
                                          result.get("cpu_baseline"))
        result["e2e_dropin_device_frames"] = e2e_dropin(es, width, height, cf, parsed.npics, device,
                                                        result.get("cpu_baseline"), device_frames=True)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if parity["status"] == "MISMATCH":
        sys.exit(3)


def e2e_dropin(es, width, height, cf, frames, device, cpu, device_frames=False):
    """The drop-in API end to end on the same stream: mp2v_decoder_c(config, renderer).decode(buf)
    with host frame_c frames (parse, upload, decode, D2H, display-order render callbacks), i.e.
    what a caller of the reference API sees (reference tiny_mp2v_dec.cpp:50-55 times decode()
    the same way); best of two decode() calls on one decoder, like cpu_baseline's best of 2.  PCIe-inclusive: never the bench `value`.  device_frames: the opt-in
    MP2VG_DECODER_DEVICE_FRAMES path (frames handed to the renderer in HBM, no D2H)."""
    from tiny_mp2v_dec_amd.decoder import decoder_config_t, mp2v_decoder_c
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 2)
    threads = max(2, min(share, os.cpu_count() or share, 16))
    count = [0]

    def render(frame):
        count[0] += 1

    dec = mp2v_decoder_c(decoder_config_t(width, height, cf, pictures_pool_size=24, num_threads=threads,
                                          device=device, device_frames=device_frames), render)
    runs = []
    try:
        for _ in range(2):  # best of 2, as cpu_baseline's reference runs (the host is shared)
            count[0] = 0
            t = time.perf_counter()
            dec.decode(es, len(es))
            runs.append(time.perf_counter() - t)
            if count[0] != frames:
                raise RuntimeError(f"drop-in rendered {count[0]} of {frames} frames")
    finally:
        dec.close()
    dt = min(runs)
    out = {"value": round(frames / dt, 1), "unit": "frames/s", "host_threads": threads, "frames": frames,
           "runs_frames_per_s": [round(frames / r, 1) for r in runs],
           "scope": "drop-in mp2v_decoder_c::decode() on the bench stream: host parse + record upload + "
                    + ("GPU reconstruct into device frame_c (HBM, no D2H) + render callbacks" if device_frames else
                       "GPU reconstruct + D2H into host frame_c + render callbacks")}
    if cpu:
        out["vs_cpu_baseline"] = round(out["value"] / cpu["value"], 3)
    return out


if __name__ == "__main__":
    main()

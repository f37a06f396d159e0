"""Benchmark: MPEG-2 macroblock reconstruct on MI355X (BASELINE.json metric / configs[1]).

A "step" = one pass of the hot path over one batch: the dequant + IDCT + MC + add/clip of every
picture of G closed GOPs (1080p 4:2:0, N=12, M=3 -> 12*G frames) whose pre-parsed macroblock
records are already resident in HBM.  Each rank (one per GPU) decodes its own independent GOP
stream (seed 1729 + rank): weak scaling, no data-path collective; RCCL only gathers per-frame
digests to rank 0 after the timed region (the trivial frame gather).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--gops G] [--config c2|c3|c4|c5]

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

from tiny_mp2v_dec_amd import build as _build  # noqa: E402
from tiny_mp2v_dec_amd import records as R  # noqa: E402

BASELINE_METRIC = "decoded frames/sec + GB/s vs HBM roofline, 1080p 4:2:0 @1/2/4/8 GPU; bit-exact YUV"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

CONFIGS = {
    # name: (width, height, chroma_format, generator params, description)
    "c2": (1920, 1088, 1, dict(gop_n=12, gop_m=3, leading_b=1), "1080p 4:2:0 IPB GOP=12 (N=12, M=3, closed)"),
    "c3": (1920, 1088, 2, dict(gop_n=12, gop_m=3, leading_b=1), "1080p 4:2:2 IPB GOP=12 (N=12, M=3, closed)"),
    "c4": (3840, 2160, 1, dict(gop_n=12, gop_m=3, leading_b=1), "4K 4:2:0 IPB GOP=12 (N=12, M=3, closed)"),
    "c5": (1920, 1088, 3, dict(gop_n=1, gop_m=1, mix=1, intra_coefs_min=20, intra_coefs_max=40),
           "1080p 4:4:4 I-only high bitrate (20-40 AC coefficients per block)"),
}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gops", type=int, default=64)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist

    if rank == 0:
        _build.build()
    if dist is not None:
        dist.barrier()

    width, height, cf, gparams, desc = CONFIGS[args.config]
    # c5 is I-only: one picture per "GOP", so --gops is its frame count (~60 frames; at
    # 768 frames its elementary stream would pass the 2 GB `int len` of the reference decode() API)
    gops = args.gops
    es = R.generate_es(width=width, height=height, chroma_format=cf, n_gops=gops, seed=1729 + rank, **gparams)
    parsed = R.Parsed(es, width, height, cf, threads=min(8, os.cpu_count() or 1))
    alg_bytes, parts = algorithmic_bytes(parsed)
    ctx = R.DeviceContext(width, height, cf, slots=parsed.npics, device=local_rank)
    ctx.upload(parsed.pics, parsed.mbs, parsed.coefs)

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
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # frame gather (digests) to rank 0 over RCCL, outside the timed region
    dig = ctx.digests(np.arange(parsed.npics))
    gathered = [dig]
    if dist is not None:
        import torch
        d = torch.from_numpy(dig.view(np.int64)).cuda()
        outs = [torch.empty_like(d) for _ in range(world)]
        dist.all_gather(outs, d)
        gathered = [o.cpu().numpy().view(np.uint64) for o in outs]

    traffic = profiled_traffic(args.config, gops)
    frames_total = parsed.npics * world * args.steps
    ms_per_step = elapsed * 1000.0 / args.steps
    per_launch = [x for step in kernel_ms for x in step]
    # the kernel time of a step is the device span of the batch (HIP events on the launch stream,
    # first launch start -> last launch end), which includes the gaps between its launches
    kernel_step_ms = float(np.mean(batch_ms))
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
                   "parallelism": f"gop-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic["traffic_bytes_per_step"] if traffic else None,
                     "traffic_unit": "bytes/step (HBM, PMC)", "traffic_source": traffic["source"] if traffic else None,
                     "kernel": "mp2vg::recon_kernel", "launches_per_step": len(kernel_ms[0]),
                     "avg_launch_ms": round(float(np.mean(per_launch)), 4),
                     "algorithmic_bytes_per_step": int(alg_bytes), "bytes_breakdown": parts,
                     "kernel_ms_per_step": round(kernel_step_ms, 4),
                     "sum_launch_ms_per_step": round(float(np.mean([sum(s) for s in kernel_ms])), 4)},
        "frame_digest_of_digests": int(np.bitwise_xor.reduce(np.concatenate(gathered))),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(es, width, height, cf, parsed.npics)
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""GPU: bench.py's multi-rank path executed for real on one MI355X -- two ranks launched by
torch.distributed.run share device 0 over the gloo backend (RCCL refuses two ranks on one GPU),
so everything bench.py does at N>1 except the RCCL transport runs: per-rank streams (seed
1729 + rank), max-over-ranks timing, the digest all_gather, per-rank parity against the compiled
reference's digests, and the rank-0 frame gather in display order."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo_on_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--backend", "gloo", "--gather-gops", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_batch_frames"] == 2 * line["config"]["frames_per_gpu_per_step"]
    assert line["parity"]["status"] == "bit-exact"
    assert line["parity"]["frames_checked"] == 2 * line["config"]["frames_per_gpu_per_step"]
    g = line["frame_gather"]
    assert g["verified"] and g["frames"] == 2 * 2 * 12
    assert line["value"] > 0 and line["roofline"]["frac"] > 0


def test_bench_plain_gpus_2_spawns_its_ranks_on_one_gpu():
    """The driver's form, `python bench.py --gpus 2` with no launcher: bench.py starts the two
    ranks itself (one torch.distributed.run child) and the line reports n_gpus 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "gloo", "--gops", "4", "--gather-gops", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["backend"] == "gloo"
    assert line["parity"]["status"] in ("bit-exact", "unchecked")


def test_bench_eight_ranks_c4_gloo_on_one_gpu():
    """The c4 8-GPU scaling command one step from the driver's: `python bench.py --gpus 8 --config
    c4 --gops 1 --backend gloo` spawns 8 ranks (all on GPU 0 here; one per GPU on a node), rank r
    decodes the one-GOP 4K stream of seed 1729 + r, and every rank's 12 frames are checked against
    the compiled reference's digests (tests/golden/bench_digests.npz, c4_g1_s1729..1736), then
    rank 0 gathers the first GOP of every rank in display order and checks it frame by frame."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--config", "c4", "--gops", "1",
           "--steps", "2", "--warmup", "1", "--backend", "gloo", "--gather-gops", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["config"]["backend"] == "gloo" and line["scaling"] == "weak"
    assert line["config"]["global_batch_frames"] == 8 * 12
    assert line["parity"]["status"] == "bit-exact" and line["parity"]["frames_checked"] == 8 * 12
    g = line["frame_gather"]
    assert g["verified"] and g["frames"] == 8 * 12


def test_bench_one_rank_over_rccl():
    """bench.py's nccl (= RCCL) branch executed for real: one rank under torch.distributed.run
    binds the process group to cuda:0 (device_id: eager communicator init), and the max-over-ranks
    all_reduce, the digest all_gather and the frame gather move cuda tensors over RCCL -- every
    collective of the 8-GPU scaling run, on the one MI355X a test box has."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--backend", "nccl", "--gather-gops", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["config"]["backend"] == "nccl"
    assert line["parity"]["status"] == "bit-exact"
    assert line["frame_gather"]["verified"] and line["frame_gather"]["frames"] == 2 * 12


def test_gather_helpers_over_rccl_world_1():
    """gather.max_over_ranks / gather_u64 / gather_gops on cuda tensors through a world-1 RCCL
    process group (a child process, so the test runner's own process never holds a communicator)."""
    code = r'''
import os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from tiny_mp2v_dec_amd import gather as G
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
assert G.max_over_ranks(2.5, dist, "cuda:0") == 2.5
a = np.array([1, 2**63 + 5, 7], np.uint64)
out = G.gather_u64(a, dist, "cuda:0")
assert len(out) == 1 and np.array_equal(out[0], a)
frames = {0: [torch.full((64,), k, dtype=torch.uint8, device="cuda:0") for k in range(3)],
          1: [torch.full((64,), 10 + k, dtype=torch.uint8, device="cuda:0") for k in range(2)]}
got = G.gather_gops(dist, frames, [3, 2], 64, device="cuda:0")
assert [int(f[0].item()) for f in got] == [0, 1, 2, 10, 11]
dist.destroy_process_group()
print("RCCL_OK")
'''
    env = dict(os.environ, REPO=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, r.stderr[-2000:]

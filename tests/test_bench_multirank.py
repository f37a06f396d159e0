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

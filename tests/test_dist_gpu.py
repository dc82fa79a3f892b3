"""The RCCL branch of the image-parallel path on the GPU box (one GPU): bench.py under
``torch.distributed.run`` with one rank and ``SAMQ_DIST_FORCE=1`` initialises an ``nccl`` (= RCCL)
process group, broadcasts the packed weights through it, times with the barrier + all-reduce(MAX)
it uses at N > 1, and reports the backend it saw.  (N > 1 ranks need N GPUs: the driver's run.)"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_one_rank_rccl_group():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["SAMQ_DIST_FORCE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"),
           "--gpus", "1", "--batch", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-isolated"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(REPO))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(f"\n[rccl] one-rank group: {out['dist']}, {out['value']} img/s")
    assert out["dist"]["backend"] == "nccl" and out["dist"]["world_size_seen"] == 1
    assert out["dist"]["broadcast_bytes"] > 300e6   # the packed ViT-H weights + fp16 params
    assert out["value"] > 0

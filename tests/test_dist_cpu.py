"""Image-parallel path on CPU with gloo, world_size 2: weight broadcast (bucketed, one collective
per dtype), contiguous image sharding, embedding gather."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "sam-quantization_amd"))
    from samq import dist as sdist
    from samq.synthetic import random_quant_encoder
    r, w = sdist.init_from_env("gloo")
    assert (r, w) == (rank, world)
    enc = random_quant_encoder("vit_b", device="cpu", img_size=256, depth=2, init=(rank == 0), seed=5)
    nbytes = sdist.broadcast_state(enc, src=0)
    sd = enc.state_dict()
    digest = sum(float(v.double().sum()) for v in sd.values() if v.is_floating_point()) + \
        sum(int(v.long().sum()) for v in sd.values() if not v.is_floating_point())
    lo, hi = sdist.shard(10, rank, world)
    local = torch.full((hi - lo, 3), float(rank))
    local = local[:4] if local.shape[0] >= 4 else torch.cat([local, local.new_zeros(4 - local.shape[0], 3)])
    got = sdist.gather_embeddings(local)
    q.put((rank, nbytes, digest, (lo, hi), None if got is None else got[:, 0].tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_shard_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, b0, d0, s0, g0), (r1, b1, d1, s1, g1) = res
    assert b0 == b1 > 0
    assert d0 == d1, "rank 1 weights differ from rank 0 after broadcast"
    assert s0 == (0, 5) and s1 == (5, 10)
    assert g0 == [0.0] * 4 + [1.0] * 4 and g1 is None


def test_shard_covers_everything():
    from samq.dist import shard
    for n in (0, 1, 7, 64):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))


def test_bench_launches_its_own_ranks_and_shards_the_global_batch():
    """``bench.py --gpus 2`` started bare (no torchrun env) spawns its 2 ranks as a child
    ``torch.distributed.run`` and relays ONE line from rank 0; the seeded global batch is split
    contiguously and each rank's images are exactly the single-process images of those indices;
    the packed weights reach rank 1 through the broadcast (gloo here, RCCL on the GPU box)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--backend", "gloo", "--dry-run",
                        "--batch", "3"], capture_output=True, text=True, timeout=300, env=env, cwd=str(repo))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size_seen"] == 2 and out["backend"] == "gloo"
    assert out["global_batch"] == 6
    ranks = sorted(out["ranks"], key=lambda d: d["rank"])
    assert [d["shard"] for d in ranks] == [[0, 3], [3, 6]]
    assert ranks[0]["state_checksum"] == ranks[1]["state_checksum"]
    assert ranks[1]["broadcast_bytes"] > 0
    sys.path.insert(0, str(repo))
    import bench
    ref = bench.local_images(0, 6, torch.device("cpu"), torch.float32, size=32)
    got = ranks[0]["image_checksums"] + ranks[1]["image_checksums"]
    assert got == [float(x.double().sum()) for x in ref]


def test_forced_one_rank_group_runs_the_collectives():
    """``SAMQ_DIST_FORCE=1`` under a one-rank torchrun environment initialises the process group
    (gloo here; RCCL in tests/test_dist_gpu.py) and the weight broadcast / gather go through it."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parent.parent
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), SAMQ_DIST_FORCE="1")
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "1", "--backend", "gloo", "--dry-run",
                        "--batch", "2"], capture_output=True, text=True, timeout=300, env=env, cwd=str(repo))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "gloo" and out["world_size_seen"] == 1
    assert out["ranks"][0]["broadcast_bytes"] > 0 and out["ranks"][0]["shard"] == [0, 2]

"""Image-parallel multi-GPU plumbing: one process per GPU, independent images.

The only data-path collective is ONE bucketed RCCL broadcast of the packed weights (plus the
fp16/fp32 non-quantised parameters) from rank 0 at load time; images are sharded contiguously
across ranks and never exchanged.  ``gather_embeddings`` optionally collects the outputs on rank 0.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None, force: bool | None = None):
    """``torch.distributed`` from torchrun's RANK / WORLD_SIZE / LOCAL_RANK (no-op if unset, and for
    a world of one unless ``force`` / ``SAMQ_DIST_FORCE=1``: a one-rank RCCL group runs the same
    communicator set-up and collectives as N ranks -- the single-GPU hardware check of this path)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if force is None:
        force = os.environ.get("SAMQ_DIST_FORCE", "") == "1" and "RANK" in os.environ
    if (ws <= 1 and not force) or dist.is_initialized():
        return (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def _buckets(tensors):
    by = {}
    for t in tensors:
        by.setdefault((t.dtype, t.device), []).append(t)
    return by


@torch.no_grad()
def broadcast_state(module: torch.nn.Module, src: int = 0) -> int:
    """Broadcast every parameter and persistent buffer of ``module`` from ``src`` with one
    collective per dtype (flattened buckets).  Returns the number of bytes broadcast."""
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    tensors = [t for t in module.state_dict().values() if torch.is_tensor(t)]
    total = 0
    for (dtype, dev), ts in _buckets(tensors).items():
        flat = torch.cat([t.reshape(-1) for t in ts]) if dist.get_rank() == src else \
            torch.empty(sum(t.numel() for t in ts), dtype=dtype, device=dev)
        dist.broadcast(flat, src)
        if dist.get_rank() != src:
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n
        total += flat.numel() * flat.element_size()
    return total


def shard(n_items: int, rank: int, world: int):
    """Contiguous [start, stop) share of ``n_items`` for ``rank`` (remainder to the first ranks)."""
    base, rem = divmod(n_items, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_embeddings(local: torch.Tensor, dst: int = 0):
    """Gather per-rank outputs (equal shapes) onto ``dst``; returns the concatenation there."""
    if not (dist.is_available() and dist.is_initialized()):
        return local
    parts = [torch.empty_like(local) for _ in range(dist.get_world_size())] if dist.get_rank() == dst else None
    dist.gather(local, parts, dst=dst)
    return torch.cat(parts) if parts is not None else None


def warm_up_collective(device=None) -> float:
    """One-element ``all_reduce`` before the weight broadcast: the first collective of a process
    group creates the communicator (RCCL's set-up) and waits for the slowest rank, so timing the
    broadcast after it measures the transfer alone.  Returns its seconds (0 without a group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 0.0
    import time
    on_gpu = device is not None and torch.device(device).type == "cuda"
    t0 = time.perf_counter()
    t = torch.zeros(1, device=device)
    dist.all_reduce(t)
    if on_gpu:
        torch.cuda.synchronize(device)
    return time.perf_counter() - t0

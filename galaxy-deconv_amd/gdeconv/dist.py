"""Batch sharding across GPUs of one node.

Galaxies are independent (no cross-batch term anywhere on the path), so a batch of N galaxies is
split into contiguous slices, one process per GPU (``torch.distributed`` over RCCL = backend
"nccl" on ROCm), with no collective on the data path.  The only collective is the optional final
``all_gather`` of the outputs over xGMI (``gather_batch``), issued in chunks so a caller can
overlap it with the next batch's compute.
"""
import os

import torch
import torch.distributed as dist


def shard_range(N, rank, world):
    """Contiguous [start, stop) slice of ``N`` galaxies for ``rank`` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(N, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), \
        int(os.environ.get("LOCAL_RANK", 0))


def init_process_group(backend=None):
    """Initialise from the torchrun environment (MASTER_ADDR should be 127.0.0.1 on one node)."""
    rank, world, local = env_rank_world()
    if world == 1 or dist.is_initialized():
        return rank, world, local
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def gather_batch(local, N, chunk_bytes=256 << 20):
    """All-gather per-rank output slices [n_r, ...] (n_r from ``shard_range``) into [N, ...] on
    every rank.  Uneven shards are padded to the largest slice; large outputs go in chunks of
    about ``chunk_bytes`` per rank so the xGMI transfers pipeline."""
    world = dist.get_world_size()
    sizes = [shard_range(N, r, world) for r in range(world)]
    mx = max(b - a for a, b in sizes)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    per_item = max(1, pad[0].numel() * pad.element_size())
    step = max(1, min(mx, chunk_bytes // per_item))
    out = torch.empty((N,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for c0 in range(0, mx, step):
        c1 = min(mx, c0 + step)
        parts = [torch.empty_like(pad[c0:c1]) for _ in range(world)]
        dist.all_gather(parts, pad[c0:c1].contiguous())
        for r, (a, b) in enumerate(sizes):
            n_r = b - a
            lo, hi = c0, min(c1, n_r)
            if hi > lo:
                out[a + lo:a + hi] = parts[r][: hi - lo]
    return out


__all__ = ["shard_range", "env_rank_world", "init_process_group", "gather_batch"]

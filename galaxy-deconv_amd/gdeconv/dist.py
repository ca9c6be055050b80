"""Batch sharding across GPUs of one node.

Galaxies are independent (no cross-batch term anywhere on the path), so a batch of N galaxies is
split into contiguous slices, one process per GPU (``torch.distributed`` over RCCL = backend
"nccl" on ROCm), with no collective on the data path.  The only collective is the optional final
all-gather of the outputs over xGMI (``gather_batch``: ``all_gather_into_tensor`` straight into
the result, chunked for large outputs, asynchronous on request so it overlaps the next batch's
forward).
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
    """Initialise from the torchrun environment (MASTER_ADDR should be 127.0.0.1 on one node).
    Backend: ``backend``, else $GD_DIST_BACKEND, else "nccl" (RCCL) with a GPU and "gloo" without;
    GD_DIST_BACKEND=gloo rehearses several ranks on one GPU (RCCL refuses two ranks per device)."""
    rank, world, local = env_rank_world()
    if world == 1 or dist.is_initialized():
        return rank, world, local
    if backend is None:
        backend = os.environ.get("GD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        if torch.cuda.device_count() <= local:
            raise RuntimeError(f"RCCL rank {rank} (local rank {local}) but {torch.cuda.device_count()} visible "
                               "GPU(s): RCCL needs one GPU per rank (GD_DIST_BACKEND=gloo rehearses on fewer)")
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def local_device(local):
    """The GPU of local rank ``local`` (ranks beyond the device count share GPUs round-robin: only
    for gloo rehearsals of the multi-rank path on fewer GPUs)."""
    n = torch.cuda.device_count()
    return torch.device("cuda", local % n if n else 0)


class PendingGather:
    """In-flight ``gather_batch(..., async_op=True)``: the collectives run on the process group's own
    stream (RCCL's internal stream on ROCm), so the caller's stream is free to run the next batch's
    forward meanwhile.  ``wait()`` makes the CURRENT stream wait for them, places the chunks that
    went through a staging buffer, and returns the gathered [N, ...] tensor."""

    def __init__(self, out, works, finish):
        self.out, self._works, self._finish = out, works, finish

    def wait(self):
        for w in self._works:
            w.wait()
        for f in self._finish:
            f()
        self._works, self._finish = [], []
        return self.out


def gather_batch(local, N, chunk_bytes=256 << 20, async_op=False):
    """All-gather per-rank output slices [n_r, ...] (n_r from ``shard_range``) into [N, ...] on every
    rank with ``all_gather_into_tensor`` (one buffer per collective, no per-rank tensor lists).

    Even shards (N divisible by the world size) and an output of at most ``chunk_bytes`` per rank land
    straight in the result: its rank-major layout IS all_gather_into_tensor's.  Larger outputs go in
    chunks of about ``chunk_bytes`` per rank, each gathered into a [world, chunk, ...] staging buffer
    and placed with one strided copy, so the xGMI transfers of chunk c + 1 overlap the placement of
    chunk c; uneven shards are padded to the largest slice.  ``async_op=True`` returns a
    ``PendingGather`` instead (overlap with the next batch's compute; see its ``wait``)."""
    if local.is_cuda and dist.get_backend() == "gloo":
        # gloo has no device all-gather: gather host copies, place the result on the device (the
        # multi-rank rehearsal on one GPU; RCCL's path below is the product path)
        out = gather_batch(local.cpu(), N, chunk_bytes).to(local.device)
        return PendingGather(out, [], []) if async_op else out
    world = dist.get_world_size()
    rank = dist.get_rank()
    sizes = [shard_range(N, r, world) for r in range(world)]
    mx = max(b - a for a, b in sizes)
    if local.shape[0] != sizes[rank][1] - sizes[rank][0]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} galaxies, shard_range gives "
                         f"{sizes[rank][1] - sizes[rank][0]}")
    tail = tuple(local.shape[1:])
    even = all(b - a == mx for a, b in sizes)
    src = local.contiguous()
    if not even:
        src = torch.zeros((mx,) + tail, dtype=local.dtype, device=local.device)
        src[: local.shape[0]] = local
    out = torch.empty((N,) + tail, dtype=local.dtype, device=local.device)
    per_item = max(1, (src[0].numel() if mx else 1) * src.element_size())
    step = max(1, min(max(mx, 1), chunk_bytes // per_item))
    works, finish = [], []
    if mx == 0:
        return PendingGather(out, [], []) if async_op else out
    if even and step >= mx:
        works.append(dist.all_gather_into_tensor(out, src, async_op=True))
    else:
        for c0 in range(0, mx, step):
            c1 = min(mx, c0 + step)
            stage = torch.empty((world * (c1 - c0),) + tail, dtype=local.dtype, device=local.device)
            works.append(dist.all_gather_into_tensor(stage, src[c0:c1].contiguous(), async_op=True))
            stage = stage.view((world, c1 - c0) + tail)

            def place(stage=stage, c0=c0, c1=c1):
                if even:
                    out.view((world, mx) + tail)[:, c0:c1].copy_(stage)
                    return
                for r, (a, b) in enumerate(sizes):
                    hi = min(c1, b - a)
                    if hi > c0:
                        out[a + c0:a + hi].copy_(stage[r, : hi - c0])
            finish.append(place)
    pending = PendingGather(out, works, finish)
    return pending if async_op else pending.wait()


__all__ = ["shard_range", "env_rank_world", "init_process_group", "local_device", "gather_batch", "PendingGather"]

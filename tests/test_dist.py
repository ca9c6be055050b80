"""World-size-2 gloo run of the N>1 host path on CPU: contiguous batch shards per rank, per-rank
compute (the CPU oracle stands in for the per-GPU engine here), all_gather_into_tensor of the
outputs (uneven / even shards, one collective or chunks, blocking or asynchronous) - the
reassembled result equals the single-process batch."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, "galaxy-deconv_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import admm_oracle as O
    from gdeconv.dist import gather_batch, shard_range
    from gdeconv.synth import make_batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        N = 5                                           # uneven on purpose
        obs, psf, alpha, _ = make_batch(N, 64, h=16, seed=4)  # every rank builds the same seeded batch
        a, b = shard_range(N, rank, world)
        local = O.wiener(obs[a:b], psf[a:b], alpha[a:b])
        full = gather_batch(local, N, chunk_bytes=4096)  # uneven shards, several chunks
        ref = O.wiener(obs, psf, alpha)
        ok = torch.equal(full, ref)
        # even shards: one collective straight into the result, and chunked; asynchronous form
        N2 = 6
        o2, p2, a2, _ = make_batch(N2, 64, h=16, seed=5)
        a, b = shard_range(N2, rank, world)
        loc2 = O.wiener(o2[a:b], p2[a:b], a2[a:b])
        ref2 = O.wiener(o2, p2, a2)
        ok &= torch.equal(gather_batch(loc2, N2), ref2)
        ok &= torch.equal(gather_batch(loc2, N2, chunk_bytes=4096), ref2)
        pend = gather_batch(loc2, N2, chunk_bytes=3 * 64 * 64 * 4, async_op=True)
        ok &= torch.equal(pend.wait(), ref2)
        if rank == 0:
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True

"""World-size-2 gloo run of the N>1 host path on CPU: contiguous batch shards per rank, per-rank
compute (the CPU oracle stands in for the per-GPU engine here), chunked all_gather of the
outputs - reassembled result equals the single-process batch."""
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
        full = gather_batch(local, N, chunk_bytes=4096)  # force several chunks
        if rank == 0:
            ref = O.wiener(obs, psf, alpha)
            q.put(bool(torch.equal(full, ref)))
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

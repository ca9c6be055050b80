"""Two ranks driving the HIP engine: each process runs Unrolled_ADMM's spectral path
on its contiguous shard on the box's GPU, the outputs are all-gathered (gloo over host copies: RCCL
refuses two ranks on one device), and the reassembled batch equals the single-process forward bit
for bit - the engine is batch-invariant, so sharding changes nothing."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(dev):
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    m = Unrolled_ADMM(n_iters=3, llh="Gaussian")
    m.load_state_dict(make_state_dict(m, 11))
    m = m.to(dev).eval()
    m.Z = torch.nn.Identity()
    return m


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, "galaxy-deconv_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    from gdeconv.dist import gather_batch, shard_range
    from gdeconv.synth import make_batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        N = 7                                                  # uneven shards
        obs, psf, alpha, _ = make_batch(N, 256, seed=21, device=dev)
        a, b = shard_range(N, rank, world)
        m = _model(dev)
        with torch.no_grad():
            local = m(obs[a:b], psf[a:b], alpha[a:b]).cpu()
        full = gather_batch(local, N, chunk_bytes=2 * 256 * 256 * 4)
        if rank == 0:
            with torch.no_grad():
                ref = m(obs, psf, alpha).cpu()
            q.put(bool(torch.equal(full, ref)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_drive_the_engine():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True

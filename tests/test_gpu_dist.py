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


def _bench(argv, env_extra, timeout=600):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *argv], capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=ROOT)


def test_bench_spawns_its_ranks():
    """``bench.py --gpus 2`` with no launcher starts its two ranks itself (gloo rehearsal on one GPU)
    and prints ONE line for the 2-rank job, with the all-gather timings of the multi-rank path."""
    import json
    r = _bench(["--gpus", "2", "--batch", "64", "--steps", "2", "--warmup", "1", "--no-e2e", "--no-ingest",
                "--no-cpu-baseline"], {"GD_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["ranks_seen"] == 2 and rec["config"]["backend"] == "gloo"
    assert rec["config"]["global_batch"] == 128 and rec["value"] > 0
    assert rec["gather_ms"] > 0 and rec["with_gather"]["value"] > 0
    assert rec["graphed"]["bit_identical_to_eager"]


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """RCCL needs one GPU per rank: ``--gpus N`` beyond the visible GPUs exits non-zero (no 1-rank line)."""
    n = torch.cuda.device_count() + 1
    r = _bench(["--gpus", str(n), "--batch", "8", "--steps", "1", "--warmup", "0", "--no-e2e", "--no-ingest",
                "--no-cpu-baseline", "--no-graph"], {"GD_DIST_BACKEND": "nccl"}, timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]

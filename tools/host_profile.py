"""Host cost of the eager drop-in forward at the LSST stamp size (configs[1]: 256 x 48^2, n_iters = 8,
identity denoiser): wall time per forward (host-bound: the GPU work is ~0.12 ms) and a cProfile of the
Python side.  python tools/host_profile.py [--size 48 --batch 256 --forwards 200]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import build_model  # noqa: E402
from gdeconv.synth import make_batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=48)
p.add_argument("--batch", type=int, default=256)
p.add_argument("--forwards", type=int, default=200)
a = p.parse_args()
dev = torch.device("cuda:0")
m = build_model(8, "Gaussian", dev)
m.Z = torch.nn.Identity()
obs, psf, alpha, _ = make_batch(a.batch, a.size, seed=5, device=dev)
with torch.no_grad():
    for _ in range(20):
        m(obs, psf, alpha)
    torch.cuda.synchronize()
    for rep in range(3):
        t = time.perf_counter()
        for _ in range(a.forwards):
            m(obs, psf, alpha)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.forwards
        print(f"eager forward {dt * 1e3:.4f} ms = {a.batch / dt / 1e6:.3f} M gal/s", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.forwards):
        m(obs, psf, alpha)
    torch.cuda.synchronize()
    pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())

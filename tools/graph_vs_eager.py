"""Eager vs hipGraph-replayed forward at 4096 x 256^2 (bench.py's model, identity denoiser): K eager steps
then K replays, for a kernel trace (rocprofv3 --kernel-trace) whose dispatches split in order."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from gdeconv.graphs import GraphedForward  # noqa: E402
from gdeconv.synth import make_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dev = torch.device("cuda:0")
obs, psf, alpha, _ = make_batch(N, 256, seed=1, device=dev)
m = bench.build_model(8, "Gaussian", dev)
m.Z = torch.nn.Identity()
with torch.no_grad():
    for _ in range(2):
        m(obs, psf, alpha)
    gf = GraphedForward(m, obs, psf, alpha)
    gf.replay()
    torch.cuda.synchronize()
    for name, fn in (("eager", lambda: m(obs, psf, alpha)), ("graph", gf.replay), ("eager", lambda: m(obs, psf, alpha)),
                     ("graph", gf.replay)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t) * 1e3 / K:.3f} ms/step", flush=True)

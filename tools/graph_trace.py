"""Kernel timeline of one hipGraph-replayed forward (bench.py's model, identity denoiser) at a given size:
K replays after capture, for `rocprofv3 --kernel-trace` (tools/graph_timeline.py splits the trace per replay
and prints each position's mean duration and the gap before it).

usage: python tools/graph_trace.py [K] [N] [L]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from gdeconv.graphs import GraphedForward  # noqa: E402
from gdeconv.synth import make_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
L = int(sys.argv[3]) if len(sys.argv) > 3 else 48
dev = torch.device("cuda:0")
obs, psf, alpha, _ = make_batch(N, L, seed=1, device=dev)
m = bench.build_model(8, "Gaussian", dev)
m.Z = torch.nn.Identity()
with torch.no_grad():
    gf = GraphedForward(m, obs, psf, alpha)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(K):
        gf.replay()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"{K} replays: {ev[0].elapsed_time(ev[1]) * 1e3 / K:.1f} us per forward", flush=True)

"""Reproduce the round-4 capture crash in isolation: Unrolled_ADMM(n_iters=8) at N x L^2 with the chunked
(pipelined) init, one eager forward, then GraphedForward (torch.cuda.graph capture + instantiate), then a replay
checked bit-for-bit against the eager output.  The capture-mode switch is GD_CAPTURE_PIPELINE (gd_engine.hip).

usage: python tools/capture_repro.py [N=4096] [L=160] [fused_init=0]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 160
    fi = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    from bench import build_model
    from gdeconv import _lib
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    lib = _lib.load()
    lib.gd_set_fused_init(fi)
    dev = torch.device("cuda:0")
    obs, psf, alpha, _ = make_batch(N, L, seed=5, device=dev)
    m = build_model(8, "Gaussian", dev)
    m.Z = torch.nn.Identity()
    with torch.no_grad():
        out = m(obs, psf, alpha)
    torch.cuda.synchronize()
    print(f"[repro] eager forward done ({N} x {L}^2, fused_init {fi}, GD_CAPTURE_PIPELINE="
          f"{os.environ.get('GD_CAPTURE_PIPELINE', 'default')})", flush=True)
    t = time.perf_counter()
    g = GraphedForward(m, obs, psf, alpha)
    torch.cuda.synchronize()
    print(f"[repro] captured + instantiated in {time.perf_counter() - t:.2f} s", flush=True)
    r = g.replay()
    torch.cuda.synchronize()
    print(f"[repro] replay bit-identical to eager: {bool(torch.equal(r, out))}", flush=True)


if __name__ == "__main__":
    main()

"""Golden vectors for the ill-conditioned Tikhonov-Laplacian solve at a second and third lambda, made by
running the REFERENCE itself (read-only import) on CPU in the build container (``/root/reference`` does
not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_tik.py

``models/Tikhonet.py:8-31``: x = Re IFFT2(conj(H) FFT2(y/alpha) / (|H|^2 + lam |L|^2)).  Where |H|^2 is
small the solve amplifies fp32 rounding by ~1/lam, so the reference's own fp32 output drifts from the exact
result (9e-6 normwise at 255^2, lam = 0.37, in sizes.npz).  These cases exercise that margin on new seeded
galaxies at two more lambdas instead of relying on one lucky draw: the GPU tests gate them with
``conftest.parity_gate`` (engine vs fp64 <= 1e-5; engine vs reference <= 1e-5 + reference vs fp64).
Only inputs and outputs are written - never reference source.

  tik_sizes.npz  for (H, W) in SIZES, N=1 seeded galaxy (gdeconv.synth.make_batch, PSF 48 x 48):
                 Tikhonov('Laplacian', lam) and Tikhonov('Identity', lam) on max(y, 0), lam in LAMS
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "galaxy-deconv_amd"))
sys.path.insert(0, HERE)
sys.path.insert(0, REF)

from gdeconv.synth import make_batch           # noqa: E402
import make_golden                             # noqa: E402,F401  (drops galaxy-deconv_amd from sys.path)
from models.Tikhonet import Tikhonov           # noqa: E402  (reference)

SIZES = [(255, 255), (192, 160)]
LAMS = [0.05, 2.0]


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    g = {"sizes": np.array(SIZES, dtype=np.int32), "lams": np.array(LAMS, dtype=np.float32)}
    for i, (H, W) in enumerate(SIZES):
        t = f"{H}x{W}"
        obs, psf, alpha, _ = make_batch(1, H, W, h=48, seed=900 + i)
        g[f"{t}_obs"], g[f"{t}_psf"], g[f"{t}_alpha"] = obs.numpy(), psf.numpy(), alpha.numpy()
        yp = torch.max(obs, torch.zeros_like(obs))
        with torch.no_grad():
            for lam in LAMS:
                for filt in ("Identity", "Laplacian"):
                    g[f"{t}_tik_{filt}_{lam}"] = Tikhonov(filter=filt)(yp, psf, alpha, torch.tensor(lam)).numpy()
    np.savez_compressed(os.path.join(HERE, "tik_sizes.npz"), **g)
    print("tik_sizes.npz", os.path.getsize(os.path.join(HERE, "tik_sizes.npz")))


if __name__ == "__main__":
    main()

"""Golden vectors at image sizes outside the compile-time-planned set (square 32/48/64/96/128/256),
made by running the REFERENCE itself (read-only import) on CPU in the build container
(``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_sizes.py

The reference's torch.fft path works for any H x W (utils/utils_torch.py:22-27, 46-50, 79-92), so the
engine's runtime-planned kernels (csrc/gd_generic.hpp) are pinned here.  Only inputs and outputs are
written - never reference source.

  sizes.npz  for each (H, W, h) in SIZES, N=2 seeded galaxies (gdeconv.synth.make_batch): conv_fft_batch
             with H and conj(H) from psf_to_otf; Wiener; Richard_Lucy(10); Unrolled_ADMM(n=4) with
             denoiser = identity for both llh (SubNet with the seed-1234 weights) and its rhos;
             Tikhonov('Identity' | 'Laplacian', lam=0.37) on max(y, 0).  Also, at 45 x 60, the full
             Unrolled_ADMM(n=2, 'Gaussian') with the ResUNet; at 40 x 40 (PSF 40 x 40),
             UnrolledADMMGaussian(n=4) with denoiser = identity.
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
from gdeconv.weights import make_state_dict    # noqa: E402
from make_golden import Identity, run_admm     # noqa: E402  (drops galaxy-deconv_amd from sys.path)
from models.Richard_Lucy import Richard_Lucy   # noqa: E402  (reference)
from models.Tikhonet import Tikhonov           # noqa: E402  (reference)
from models.Unrolled_ADMM import Unrolled_ADMM  # noqa: E402  (reference)
from models.unrolled_admm_gaussian import UnrolledADMMGaussian  # noqa: E402  (reference)
from models.Wiener import Wiener               # noqa: E402  (reference)
from utils.utils_torch import conv_fft_batch, psf_to_otf  # noqa: E402  (reference)

WEIGHT_SEED = 1234
# (H, W, psf side): a radix-2/5 square, a non-square pair, an odd side, a prime side, radix 3 and 5,
# odd widths
SIZES = [(40, 40, 32), (64, 48, 32), (45, 60, 32), (97, 80, 48), (192, 160, 48),
         (45, 61, 32), (255, 255, 48)]  # odd W (no Nyquist column): 61 prime, 255 = 3 5 17
LAM = 0.37


def tag(H, W):
    return f"{H}x{W}"


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    g = {"sizes": np.array(SIZES, dtype=np.int32)}
    for i, (H, W, h) in enumerate(SIZES):
        t = tag(H, W)
        obs, psf, alpha, _ = make_batch(2, H, W, h=h, seed=500 + i)
        g[f"{t}_obs"], g[f"{t}_psf"], g[f"{t}_alpha"] = obs.numpy(), psf.numpy(), alpha.numpy()
        _, Hk = psf_to_otf(psf, obs.size())
        g[f"{t}_conv_H"] = conv_fft_batch(Hk, obs).numpy()
        g[f"{t}_conv_Ht"] = conv_fft_batch(torch.conj(Hk), obs).numpy()
        with torch.no_grad():
            g[f"{t}_wiener"] = Wiener()(obs, psf, alpha).numpy()
            g[f"{t}_rl10"] = Richard_Lucy(10)(obs, psf).numpy()
            yp = torch.max(obs, torch.zeros_like(obs))
            for filt in ("Identity", "Laplacian"):
                g[f"{t}_tik_{filt}"] = Tikhonov(filter=filt)(yp, psf, alpha, torch.tensor(LAM)).numpy()
        for llh in ("Gaussian", "Poisson"):
            r = run_admm(obs, psf, alpha, 4, llh, identity=True)
            for k, v in r.items():
                g[f"{t}_{llh}_{k}"] = v
    # the full model (SubNet + ResUNet, seed-1234 weights) at an odd, non-square size
    obs, psf, alpha, _ = make_batch(2, 45, 60, h=32, seed=600)
    g["full_obs"], g["full_psf"], g["full_alpha"] = obs.numpy(), psf.numpy(), alpha.numpy()
    r = run_admm(obs, psf, alpha, 2, "Gaussian")
    g["full_out"] = r["out"]
    # UnrolledADMMGaussian (2x padded grid 80 x 80), identity denoiser
    obs, psf, alpha, _ = make_batch(2, 40, 40, h=40, seed=601)
    m = UnrolledADMMGaussian(n_iters=4, subnet=True, analysis=True)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    m.eval()
    m.Z = Identity()
    with torch.no_grad():
        g["gx_rho"] = m.init(psf, alpha).numpy()
        g["gx_out"] = m(obs, psf, alpha)[1][-1].numpy()
    g["gx_obs"], g["gx_psf"], g["gx_alpha"] = obs.numpy(), psf.numpy(), alpha.numpy()
    np.savez_compressed(os.path.join(HERE, "sizes.npz"), **g)
    print("sizes.npz", os.path.getsize(os.path.join(HERE, "sizes.npz")))


if __name__ == "__main__":
    main()

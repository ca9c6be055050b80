"""Golden vectors of UnrolledADMMGaussian on NON-SQUARE images, made by running the REFERENCE itself
(read-only import) on CPU in the build container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_gx_rect.py

models/unrolled_admm_gaussian.py:117-152 pads the image and its image-size kernel per axis
(pad_double, utils/utils_torch.py:11-13), so H != W runs on a 2H x 2W grid.  Only inputs and outputs
are written - never reference source.

  gauss2x_rect.npz  for each (H, W) in SIZES, N=2 seeded galaxies (gdeconv.synth.make_batch, PSF H x W):
                    the SubNet's rhos (seed-1234 weights) and the forward's last x and z
                    (UnrolledADMMGaussian(n=4, analysis=True) with denoiser = identity), and init_l2's z0.
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
from make_golden import Identity               # noqa: E402  (drops galaxy-deconv_amd from sys.path)
from models.unrolled_admm_gaussian import UnrolledADMMGaussian  # noqa: E402  (reference)
from utils.utils_torch import pad_double       # noqa: E402  (reference)

WEIGHT_SEED = 1234
SIZES = [(40, 56), (48, 30)]  # 80 x 112 and 96 x 60 grids (runtime-planned; 60 = 4 3 5)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    g = {"sizes": np.array(SIZES, dtype=np.int32)}
    fs = torch.fft
    for i, (H, W) in enumerate(SIZES):
        t = f"{H}x{W}"
        obs, _, alpha, _ = make_batch(2, H, W, h=min(H, W), seed=700 + i)
        # an H x W kernel (the model pads the kernel like the image): a normalised elliptical Gaussian
        yy, xx = torch.meshgrid(torch.arange(H) - H / 2 + 0.5, torch.arange(W) - W / 2 + 0.5, indexing="ij")
        s = torch.tensor([1.7, 2.3]).view(2, 1, 1)
        psf = torch.exp(-(yy ** 2 / (2 * s ** 2) + xx ** 2 / (2 * (1.4 * s) ** 2)))
        psf = (psf / psf.sum(dim=(-2, -1), keepdim=True)).unsqueeze(1).float()
        m = UnrolledADMMGaussian(n_iters=4, subnet=True, analysis=True)
        m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
        m.eval()
        m.Z = Identity()
        with torch.no_grad():
            g[f"{t}_rho"] = m.init(psf, alpha).numpy()
            xs, zs, us, _ = m(obs, psf, alpha)
            y = torch.maximum(obs, torch.zeros_like(obs))
            Y = fs.fft2(fs.ifftshift(pad_double(y), dim=(-2, -1)))
            Hk = fs.fft2(fs.ifftshift(pad_double(psf), dim=(-2, -1)))
            g[f"{t}_z0"] = m.init_l2(Y, torch.conj(Hk), torch.abs(Hk) ** 2, alpha).numpy()
        g[f"{t}_x"] = xs[-1].numpy()
        g[f"{t}_out"] = zs[-1].numpy()
        g[f"{t}_obs"], g[f"{t}_psf"], g[f"{t}_alpha"] = obs.numpy(), psf.numpy(), alpha.numpy()
    np.savez_compressed(os.path.join(HERE, "gauss2x_rect.npz"), **g)
    print("gauss2x_rect.npz", os.path.getsize(os.path.join(HERE, "gauss2x_rect.npz")))


if __name__ == "__main__":
    main()

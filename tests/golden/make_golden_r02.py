"""Round-2 golden vectors, made by running the REFERENCE itself (read-only import) on CPU in the build
container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r02.py

Only inputs and outputs are written - never reference source.

  admm_xdense48.npz  Unrolled_ADMM(n_iters=2, denoiser='XDenseUNet') (models/Unrolled_ADMM.py:142-151,
                     :163) for llh in {Gaussian, Poisson} at 48^2 (N=2: tutorial stamp + seeded), the
                     deterministic weights of gdeconv.weights (seed 1234), eval mode; the model's
                     state_dict keys are stored too (the drop-in must match them).
"""
import json
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

from gdeconv.weights import make_state_dict    # noqa: E402
from make_golden import batch48                # noqa: E402  (drops galaxy-deconv_amd from sys.path)
from models.Unrolled_ADMM import Unrolled_ADMM  # noqa: E402  (reference)

WEIGHT_SEED = 1234


def xdense_fixtures():
    obs, psf, alpha = batch48()
    g = {"obs": obs.numpy(), "psf": psf.numpy(), "alpha": alpha.numpy()}
    keys = None
    for llh in ("Gaussian", "Poisson"):
        m = Unrolled_ADMM(n_iters=2, llh=llh, denoiser="XDenseUNet", PnP=True, subnet=True)
        m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
        m.eval()
        with torch.no_grad():
            g[f"{llh}_out"] = m(obs, psf, alpha).numpy().astype(np.float32)
        keys = {k: list(v.shape) for k, v in m.state_dict().items()}
    g["state_dict_keys"] = np.frombuffer(json.dumps(keys, sort_keys=True).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "admm_xdense48.npz"), **g)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    xdense_fixtures()
    print("admm_xdense48.npz", os.path.getsize(os.path.join(HERE, "admm_xdense48.npz")))


if __name__ == "__main__":
    main()

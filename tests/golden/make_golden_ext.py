"""Golden vectors for the SURVEY 8(f) rows, made by running the REFERENCE itself (read-only import)
on CPU in the build container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ext.py

Only inputs and outputs are written - never reference source.

  tikhonov.npz   Tikhonov('Identity'|'Laplacian') (models/Tikhonet.py:8-31) at 48^2 (N=2: tutorial
                 stamp + seeded) and 256^2 (N=1), lam in {1.0, 0.37}, applied to max(y, 0) as
                 Tikhonet does; Tikhonet (models/Tikhonet.py:34-47, XDenseUNet with the
                 deterministic weights of gdeconv.weights seed 1234) at 48^2, both filters.
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
from make_golden import batch48                # noqa: E402  (drops galaxy-deconv_amd from sys.path)
from models.Tikhonet import Tikhonet, Tikhonov  # noqa: E402  (reference)

WEIGHT_SEED = 1234
LAMS = (1.0, 0.37)


def tikhonov_fixtures():
    g = {}
    o256, p256, a256, _ = make_batch(1, 256, seed=13)
    for tag, (o, p, a) in {"48": batch48(), "256": (o256, p256, a256)}.items():
        g[f"obs{tag}"], g[f"psf{tag}"], g[f"alpha{tag}"] = o.numpy(), p.numpy(), a.numpy()
        yp = torch.max(o, torch.zeros_like(o))
        for filt in ("Identity", "Laplacian"):
            t = Tikhonov(filter=filt)
            for lam in LAMS:
                with torch.no_grad():
                    g[f"tik_{filt}_{lam}_{tag}"] = t(yp, p, a, torch.tensor(lam)).numpy()
    o, p, a = batch48()
    for filt in ("Identity", "Laplacian"):
        m = Tikhonet(filter=filt)
        m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
        m.eval()
        with torch.no_grad():
            g[f"tikhonet_{filt}_48"] = m(o, p, a).numpy()
    np.savez_compressed(os.path.join(HERE, "tikhonov.npz"), **g)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    tikhonov_fixtures()
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()

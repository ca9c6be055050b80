"""Golden vectors for the SURVEY 8(f) rows, made by running the REFERENCE itself (read-only import)
on CPU in the build container (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ext.py

Only inputs and outputs are written - never reference source.

  tikhonov.npz   Tikhonov('Identity'|'Laplacian') (models/Tikhonet.py:8-31) at 48^2 (N=2: tutorial
                 stamp + seeded) and 256^2 (N=1), lam in {1.0, 0.37}, applied to max(y, 0) as
                 Tikhonet does; Tikhonet (models/Tikhonet.py:34-47, XDenseUNet with the
                 deterministic weights of gdeconv.weights seed 1234) at 48^2, both filters.
  gauss2x.npz    UnrolledADMMGaussian (models/unrolled_admm_gaussian.py:96-152) at 48^2 (N=2):
                 full model n=2 and n=8 (SubNet + ResUNet nc=32..256, seed-1234 weights, eval) with
                 analysis traces x/z/u and the SubNet rhos; identity denoiser n=8; gradients of
                 loss = sum(out * R) (R seeded) w.r.t. rho_iters (subnet=False, identity denoiser,
                 n=4) and w.r.t. four parameters of the full model (n=2); identity-denoiser outputs
                 at 32^2 and 64^2 (N=1).
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
from models.unrolled_admm_gaussian import UnrolledADMMGaussian  # noqa: E402  (reference)

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


class Identity(torch.nn.Module):
    def forward(self, z):
        return z


GRAD_KEYS = ("init.mlp.4.weight", "init.mlp.4.bias", "Z.net.m_tail.weight", "Z.net.m_head.weight")


def gauss2x_model(n, identity=False, subnet=True):
    m = UnrolledADMMGaussian(n_iters=n, subnet=subnet, analysis=True)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    m.eval()
    if identity:
        m.Z = Identity()
    return m


def gauss2x_fixtures():
    o, p, a = batch48()
    g = {"obs": o.numpy(), "psf": p.numpy(), "alpha": a.numpy()}
    for n in (2, 8):
        m = gauss2x_model(n)
        with torch.no_grad():
            g[f"full_n{n}_rho"] = m.init(p, a).numpy()
            xs, zs, us, _ = m(o, p, a)
        g[f"full_n{n}_out"] = zs[-1].numpy()
        for k, lst in (("x", xs), ("z", zs), ("u", us)):
            g[f"full_n{n}_{k}"] = torch.stack(lst).numpy()
    m = gauss2x_model(8, identity=True)
    with torch.no_grad():
        g["id_n8_rho"] = m.init(p, a).numpy()
        g["id_n8_out"] = m(o, p, a)[1][-1].numpy()
    R = torch.randn(o.shape, generator=torch.Generator().manual_seed(99))
    g["R"] = R.numpy()
    # gradients, identity denoiser, subnet=False (rho_iters parameter)
    m = gauss2x_model(4, identity=True, subnet=False)
    m.train()
    m.rho_iters.grad = None
    out = m(o, p, a)[1][-1]
    (out * R).sum().backward()
    g["grad_rho_iters"] = m.rho_iters.detach().numpy()
    g["grad_rho_iters_out"] = out.detach().numpy()
    g["grad_rho_iters_grad"] = m.rho_iters.grad.numpy()
    # gradients through SubNet + ResUNet (eval-mode BN), n=2
    m = gauss2x_model(2)
    out = m(o, p, a)[1][-1]
    (out * R).sum().backward()
    params = dict(m.named_parameters())
    g["grad_full_out"] = out.detach().numpy()
    for k in GRAD_KEYS:
        g[f"grad_full_{k}"] = params[k].grad.numpy()
    for L in (32, 64):
        o1, p1, a1, _ = make_batch(1, L, h=L, seed=40 + L)
        m = gauss2x_model(8, identity=True)
        with torch.no_grad():
            g[f"id{L}_obs"], g[f"id{L}_psf"], g[f"id{L}_alpha"] = o1.numpy(), p1.numpy(), a1.numpy()
            g[f"id{L}_rho"] = m.init(p1, a1).numpy()
            g[f"id{L}_out"] = m(o1, p1, a1)[1][-1].numpy()
    np.savez_compressed(os.path.join(HERE, "gauss2x.npz"), **g)


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    tikhonov_fixtures()
    gauss2x_fixtures()
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()

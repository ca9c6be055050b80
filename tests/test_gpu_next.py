"""GPU parity for the SURVEY 8(f) rows built on the engine: Tikhonov / Tikhonet
(models/Tikhonet.py).  Bar: per galaxy max|out - ref| <= 1e-5 * max|ref| (fp32), against the
reference's golden vectors (tests/golden/make_golden_ext.py) and the oracle."""
import numpy as np
import pytest
import torch

import admm_oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

TOL = 1e-5
WEIGHT_SEED = 1234


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def nerr(out, ref):
    return float(O.normwise_error(out, ref).max())


@pytest.mark.parametrize("tag", ["48", "256"])
@pytest.mark.parametrize("filt", ["Identity", "Laplacian"])
def test_tikhonov(dev, tag, filt):
    from gdeconv.models import Tikhonov
    g = golden("tikhonov.npz")
    obs, psf, alpha = T(g[f"obs{tag}"]), T(g[f"psf{tag}"]), T(g[f"alpha{tag}"])
    yp = torch.max(obs, torch.zeros_like(obs))
    t = Tikhonov(filter=filt)
    for lam in (1.0, 0.37):
        out = t(yp.to(dev), psf.to(dev), alpha.to(dev), torch.tensor(lam)).cpu()
        assert nerr(out, T(g[f"tik_{filt}_{lam}_{tag}"])) < TOL
        assert nerr(out, O.tikhonov(yp, psf, alpha, torch.tensor(lam), filt)) < TOL


def test_filter_power_of_placed_laplacian(dev):
    from gdeconv import engine
    from gdeconv.models import laplacian_kernel, placed_filter
    for L in (48, 256):
        img = placed_filter(laplacian_kernel(), L, L, dev)
        ltl = engine.filter_power(img).cpu()[0]                          # [K, L] (kx, ky)
        _, Lf = O.psf_to_otf(O.laplacian_kernel().double(), (1, 1, L, L), dtype=torch.float64)
        ref = (Lf.abs() ** 2)[0, 0, :, : L // 2 + 1].T                  # [K, L]
        assert float(((ltl.double() - ref).abs().max() / ref.abs().max())) < 2e-6


@pytest.mark.parametrize("filt", ["Identity", "Laplacian"])
def test_tikhonet_drop_in(dev, filt):
    from gdeconv.weights import make_state_dict
    from models.Tikhonet import Tikhonet
    g = golden("tikhonov.npz")
    obs, psf, alpha = T(g["obs48"]), T(g["psf48"]), T(g["alpha48"])
    m = Tikhonet(filter=filt)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    m = m.to(dev).eval()
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert nerr(out, T(g[f"tikhonet_{filt}_48"])) < TOL


def test_tikhonov_per_galaxy_lambda(dev):
    from gdeconv import engine
    g = golden("tikhonov.npz")
    obs, psf, alpha = T(g["obs48"]), T(g["psf48"]), T(g["alpha48"])
    lam = torch.tensor([1.0, 0.37])
    out = engine.tikhonov(obs.to(dev), psf.to(dev), alpha.to(dev), lam.to(dev)).cpu()
    for i, lv in enumerate((1.0, 0.37)):
        ref = O.tikhonov(obs[i:i + 1], psf[i:i + 1], alpha[i:i + 1], torch.tensor(lv))
        assert nerr(out[i:i + 1], ref) < TOL

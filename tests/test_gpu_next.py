"""GPU parity for the SURVEY 8(f) rows built on the engine: Tikhonov / Tikhonet
(models/Tikhonet.py).  Bar: per galaxy max|out - ref| <= 1e-5 * max|ref| (fp32), against the
reference's golden vectors (tests/golden/make_golden_ext.py) and the oracle."""
import numpy as np
import pytest
import torch

import admm_oracle as O
from conftest import golden, parity_gate

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
        ref64 = O.tikhonov(yp.double(), psf.double(), alpha.double(), torch.tensor(lam, dtype=torch.float64), filt)
        parity_gate(f"Tikhonov({filt}, lam={lam}) {tag}^2", out, T(g[f"tik_{filt}_{lam}_{tag}"]), ref64)


def test_filter_power_of_placed_laplacian(dev):
    from gdeconv import engine
    from gdeconv.models import laplacian_kernel, placed_filter
    for L in (48, 256):
        img = placed_filter(laplacian_kernel(), L, L, dev)
        ltl = engine.filter_power(img).cpu()[0]                          # [K, L] (kx, ky)
        _, Lf = O.psf_to_otf(O.laplacian_kernel().double(), (1, 1, L, L), dtype=torch.float64)
        ref = (Lf.abs() ** 2)[0, 0, :, : L // 2 + 1].T                  # [K, L]
        assert float(((ltl.double() - ref).abs().max() / ref.abs().max())) < 2e-6
        taps = engine.filter_power_taps(placed_filter(laplacian_kernel(), L, L, "cpu"), dev).cpu()[0]
        assert float(((taps.double() - ref).abs() / ref.abs().clamp_min(1e-30)).max()) < 1e-6


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


# ------------------------------------------------------------------ UnrolledADMMGaussian (8(f) row 1)
class FixedRho(torch.nn.Module):
    def __init__(self, rho):
        super().__init__()
        self.rho = rho

    def forward(self, kernel, alpha):
        return self.rho.to(kernel.device)


def _gx_model(n, dev, identity=False, subnet=True, analysis=False):
    from gdeconv.weights import make_state_dict
    from models.unrolled_admm_gaussian import UnrolledADMMGaussian
    m = UnrolledADMMGaussian(n_iters=n, subnet=subnet, analysis=analysis)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    if identity:
        m.Z = torch.nn.Identity()
    return m.to(dev).eval()


@pytest.mark.parametrize("case", ["48", "32", "64"])
def test_gauss2x_identity_denoiser(dev, case):
    g = golden("gauss2x.npz")
    pre = "" if case == "48" else f"id{case}_"
    obs, psf, alpha = T(g[pre + "obs"]), T(g[pre + "psf"]), T(g[pre + "alpha"])
    rho, ref = (T(g["id_n8_rho"]), T(g["id_n8_out"])) if case == "48" else (T(g[pre + "rho"]), T(g[pre + "out"]))
    m = _gx_model(8, dev, identity=True)
    m.init = FixedRho(rho)
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert nerr(out, ref) < TOL
    assert nerr(out, O.gx_forward(obs, psf, alpha, rho)) < TOL


@pytest.mark.parametrize("n", [2, 8])
def test_gauss2x_full_model_drop_in(dev, n):
    """Fused no-grad path (X update + dual update + next denoiser input in one engine call)."""
    g = golden("gauss2x.npz")
    obs, psf, alpha = (T(g[k]).to(dev) for k in ("obs", "psf", "alpha"))
    m = _gx_model(n, dev)
    with torch.no_grad():
        out = m(obs, psf, alpha).cpu()
    assert nerr(out, T(g[f"full_n{n}_out"])) < TOL


def test_gauss2x_analysis_traces(dev):
    g = golden("gauss2x.npz")
    obs, psf, alpha = (T(g[k]).to(dev) for k in ("obs", "psf", "alpha"))
    m = _gx_model(8, dev, analysis=True)
    with torch.no_grad():
        xs, zs, us, rhos = m(obs, psf, alpha)
    for k, lst in (("x", xs), ("z", zs), ("u", us)):
        ref = T(g[f"full_n8_{k}"])
        for i, t in enumerate(lst):
            assert nerr(t.cpu(), ref[i]) < TOL, (k, i)


def test_gauss2x_grad_rho_iters(dev):
    """Training path: HIP backward of the X update (subnet=False, identity denoiser, n=4)."""
    g = golden("gauss2x.npz")
    obs, psf, alpha, R = (T(g[k]).to(dev) for k in ("obs", "psf", "alpha", "R"))
    m = _gx_model(4, dev, identity=True, subnet=False)
    with torch.no_grad():
        m.rho_iters.copy_(T(g["grad_rho_iters"]))
    m.train()
    out = m(obs, psf, alpha)
    (out * R).sum().backward()
    assert nerr(out.detach().cpu(), T(g["grad_rho_iters_out"])) < TOL
    ref = T(g["grad_rho_iters_grad"])
    assert float((m.rho_iters.grad.cpu() - ref).abs().max() / ref.abs().max()) < TOL


def test_gauss2x_grad_full_model(dev):
    """Gradients through SubNet (eval BN) + ResUNet + HIP X-update backward, n=2."""
    g = golden("gauss2x.npz")
    obs, psf, alpha, R = (T(g[k]).to(dev) for k in ("obs", "psf", "alpha", "R"))
    m = _gx_model(2, dev)
    out = m(obs, psf, alpha)
    (out * R).sum().backward()
    assert nerr(out.detach().cpu(), T(g["grad_full_out"])) < TOL
    params = dict(m.named_parameters())
    for k in ("init.mlp.4.weight", "init.mlp.4.bias", "Z.net.m_tail.weight", "Z.net.m_head.weight"):
        ref = T(g[f"grad_full_{k}"])
        got = params[k].grad.cpu()
        assert float((got - ref).abs().max() / ref.abs().max()) < 1e-4, k


def test_gauss2x_x_update_adjoint(dev):
    """<M a, b> = <a, M b> for the X update's linear part, and d/drho against a central difference."""
    from gdeconv import engine
    g = golden("gauss2x.npz")
    obs, psf, alpha = (T(g[k]).to(dev) for k in ("obs", "psf", "alpha"))
    st = engine.GaussXState(obs, psf, alpha)
    gen = torch.Generator().manual_seed(5)
    a, b, u = (torch.randn(obs.shape, generator=gen).to(dev) for _ in range(3))
    rho = torch.tensor([0.7, 1.3], device=dev).view(2, 1, 1, 1)
    zero = torch.zeros_like(obs)
    base = st.x_update(zero, zero, rho)[0]
    Ma = st.x_update(a, zero, torch.ones(1, device=dev))[0] - st.x_update(zero, zero, torch.ones(1, device=dev))[0]
    Mb = st.x_update(b, zero, torch.ones(1, device=dev))[0] - st.x_update(zero, zero, torch.ones(1, device=dev))[0]
    lhs, rhs = float((Ma * b).sum()), float((a * Mb).sum())
    assert abs(lhs - rhs) <= 1e-5 * max(abs(lhs), abs(rhs))
    # gradients against autograd through the fp64 oracle (models/unrolled_admm_gaussian.py:89-93)
    z = a.clone().requires_grad_(True)
    r = rho.clone().requires_grad_(True)
    uu = u.clone().requires_grad_(True)
    x = engine.gx_x_update(st, z, uu, r)
    (x * b).sum().backward()
    y64, Y, Ht, HtH = O.gx_spectra(obs.cpu().double(), psf.cpu().double())
    z64 = a.cpu().double().requires_grad_(True)
    u64 = u.cpu().double().requires_grad_(True)
    r64 = rho.cpu().double().requires_grad_(True)
    x64 = O.gx_x_update(Y, Ht, HtH, z64, u64, r64)
    assert nerr(x.detach().cpu(), x64.detach()) < TOL
    (x64 * b.cpu().double()).sum().backward()
    assert nerr(z.grad.cpu(), z64.grad) < TOL
    assert nerr(uu.grad.cpu(), u64.grad) < TOL
    assert float(((r.grad.cpu().double() - r64.grad).abs() / r64.grad.abs()).max()) < TOL
    del base

"""GPU parity of the runtime-planned path (csrc/gd_generic.hpp): image sizes outside the compile-time
set (square 32/48/64/96/128/256), square or not, odd, prime, up to 1024 per side - against the
reference's golden vectors (tests/golden/make_golden_sizes.py) and the oracle; up to 4096 per side against the fp64
oracle (lines longer than 1638 points take the CU's whole 160 KiB of LDS).
Bar: per galaxy max|out - ref| <= 1e-5 * max|ref| (fp32)."""
import numpy as np
import pytest
import torch

import admm_oracle as O
from conftest import golden, parity_gate

pytestmark = pytest.mark.gpu

TOL = 1e-5
SIZES = [(40, 40), (64, 48), (45, 60), (97, 80), (192, 160), (45, 61), (255, 255)]   # sizes.npz (odd W last)
FFT_SIZES = [(2, 2), (3, 5), (17, 19), (40, 40), (64, 48), (45, 60), (97, 80), (243, 125), (1000, 30),
             (7, 1024), (1024, 1024), (96, 256), (256, 255), (1638, 1200), (1536, 1638), (1025, 1637),
             (1639, 1640), (2053, 3000), (4096, 4096)]   # lines > 1638: the 160 KiB LDS budget (round 6)


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def nerr(out, ref):
    return float(O.normwise_error(out, ref).max())


def report(tag, out, ref):
    import json
    import os
    e = nerr(out, ref)
    pix = float(O.pixel_error_floored(out, ref).max())
    print(f"[parity] {tag}: normwise {e:.3e}, per-pixel (floor 1e-5 max|ref|) {pix:.3e}")
    log = os.environ.get("GD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"case": tag, "normwise": e, "per_pixel_floored": pix}) + "\n")
    return e


@pytest.fixture(scope="module")
def eng(dev):
    from gdeconv import engine
    return engine


def load(H, W):
    g = golden("sizes.npz")
    t = f"{H}x{W}"
    return g, t, T(g[f"{t}_obs"]), T(g[f"{t}_psf"]), T(g[f"{t}_alpha"])


@pytest.mark.parametrize("H,W", FFT_SIZES)
def test_generic_rfft2_matches_fp64(eng, dev, H, W):
    from gdeconv import _lib
    assert _lib.load().gd_supported_size(H, W) == (1 if H == W and H in (32, 48, 64, 96, 128, 256) else 2)
    N = 2 if H * W <= 65536 else 1
    x = torch.randn(N, 1, H, W, generator=torch.Generator().manual_seed(H * 7 + W))
    spec = eng.rfft2_half(x.to(dev)).cpu()                       # [N, K, H] (kx, ky)
    ref = torch.fft.rfft2(x.double())[:, 0].transpose(1, 2)
    e = (spec.to(torch.complex128) - ref).abs().amax((1, 2)) / ref.abs().amax((1, 2))
    print(f"rfft2 {H}x{W}: {float(e.max()):.2e}")
    assert float(e.max()) < 3e-6
    back = eng.irfft2_half(spec.to(dev), H, W).cpu()
    assert nerr(back, x) < 3e-6


@pytest.mark.parametrize("H,W", SIZES)
def test_generic_conv_and_psf_to_otf(eng, dev, H, W):
    g, t, obs, psf, _ = load(H, W)
    otf = eng.psf_to_otf_half(psf.to(dev), 2, H, W)
    _, Href = O.psf_to_otf(psf, obs.size())
    ref_half = Href[:, 0, :, : W // 2 + 1].transpose(1, 2)
    assert nerr(torch.view_as_real(otf.cpu()), torch.view_as_real(ref_half)) < TOL
    assert report(f"conv_fft_batch {t}", eng.conv_half(otf, obs.to(dev)).cpu(), T(g[f"{t}_conv_H"])) < TOL
    assert nerr(eng.conv_half(otf, obs.to(dev), conj=True).cpu(), T(g[f"{t}_conv_Ht"])) < TOL
    # one shared OTF broadcast over the batch (fftn(x) * H with H [1,1,H,W])
    out = eng.conv_half(otf[:1], obs.to(dev)).cpu()
    assert nerr(out, O.conv_fft_batch(Href[:1], obs)) < TOL


@pytest.mark.parametrize("H,W", SIZES)
def test_generic_reference_layout_helpers(dev, H, W):
    from utils.utils_torch import conv_fft_batch, psf_to_otf
    g, t, obs, psf, _ = load(H, W)
    kpad, Hk = psf_to_otf(psf.to(dev), obs.size())
    kref, Href = O.psf_to_otf(psf, obs.size())
    assert torch.equal(kpad.cpu(), kref)
    assert nerr(torch.view_as_real(Hk.cpu()), torch.view_as_real(Href)) < TOL
    assert nerr(conv_fft_batch(Hk, obs.to(dev)).cpu(), T(g[f"{t}_conv_H"])) < TOL


@pytest.mark.parametrize("H,W", SIZES)
def test_generic_wiener_rl_tikhonov(dev, H, W):
    from gdeconv.models import Tikhonov
    from models.Richard_Lucy import Richard_Lucy
    from models.Wiener import Wiener
    g, t, obs, psf, alpha = load(H, W)
    o, p, a = obs.to(dev), psf.to(dev), alpha.to(dev)
    od, pd, ad = obs.double(), psf.double(), alpha.double()
    # engine-limited gates (conftest.parity_gate): Tikhonov-Laplacian at 255^2 has the reference's own fp32
    # output 9e-6 from the exact result, so engine-vs-reference alone would gate on the reference's rounding
    parity_gate(f"Wiener {t}", Wiener()(o, p, a).cpu(), T(g[f"{t}_wiener"]), O.wiener(od, pd, ad))
    parity_gate(f"Richard_Lucy(10) {t}", Richard_Lucy(10)(o, p).cpu(), T(g[f"{t}_rl10"]),
                O.richardson_lucy(od, pd, 10))
    yp = torch.clamp_min(o, 0)
    for filt in ("Identity", "Laplacian"):
        out = Tikhonov(filter=filt)(yp, p, a, torch.tensor(0.37)).cpu()
        parity_gate(f"Tikhonov({filt}) {t}", out, T(g[f"{t}_tik_{filt}"]),
                    O.tikhonov(yp.cpu().double(), pd, ad, torch.tensor(0.37, dtype=torch.float64), filt))


@pytest.mark.parametrize("H,W", [(255, 255), (192, 160)])
def test_generic_tikhonov_second_lambdas(dev, H, W):
    """Tikhonov-Laplacian / Identity at lam 0.05 and 2.0 on new seeded galaxies (tik_sizes.npz): the
    ill-conditioned solve's margin exercised at more than one draw, gated engine-limited."""
    from gdeconv.models import Tikhonov
    g = golden("tik_sizes.npz")
    t = f"{H}x{W}"
    obs, psf, alpha = (T(g[f"{t}_{k}"]) for k in ("obs", "psf", "alpha"))
    yp = torch.clamp_min(obs, 0)
    for lam in (0.05, 2.0):   # make_golden_tik.LAMS
        for filt in ("Identity", "Laplacian"):
            out = Tikhonov(filter=filt)(yp.to(dev), psf.to(dev), alpha.to(dev), torch.tensor(lam)).cpu()
            ref64 = O.tikhonov(yp.double(), psf.double(), alpha.double(), torch.tensor(lam, dtype=torch.float64), filt)
            parity_gate(f"Tikhonov({filt}, lam={lam}) {t}", out, T(g[f"{t}_tik_{filt}_{lam}"]), ref64)


def _spectral_model(n, llh, dev, rho1, rho2):
    from models.Unrolled_ADMM import Unrolled_ADMM
    m = Unrolled_ADMM(n_iters=n, llh=llh).to(dev).eval()
    m.Z = torch.nn.Identity()
    m.rhos = lambda k, a: (rho1.to(dev), rho2.to(dev))
    return m


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
@pytest.mark.parametrize("H,W", SIZES)
def test_generic_admm_identity_denoiser(dev, H, W, llh):
    g, t, obs, psf, alpha = load(H, W)
    m = _spectral_model(4, llh, dev, T(g[f"{t}_{llh}_rho1"]), T(g[f"{t}_{llh}_rho2"]))
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert report(f"Unrolled_ADMM(4, {llh}) identity {t}", out, T(g[f"{t}_{llh}_out"])) < TOL


def test_generic_subnet_rhos(dev):
    """The SubNet (engine feature kernel + MLP) on the PSFs of a generic-size batch: the rhos the
    reference computed for the fixture."""
    from gdeconv.weights import make_state_dict
    from models.Unrolled_ADMM import Unrolled_ADMM
    g, t, obs, psf, alpha = load(97, 80)
    m = Unrolled_ADMM(n_iters=4, llh="Gaussian")
    m.load_state_dict(make_state_dict(m, 1234))
    m = m.to(dev).eval()
    with torch.no_grad():
        r1, r2 = m.init(psf.to(dev), alpha.to(dev))
    assert nerr(r1.cpu().reshape(2, -1), T(g[f"{t}_Gaussian_rho1"]).reshape(2, -1)) < TOL
    assert nerr(r2.cpu().reshape(2, -1), T(g[f"{t}_Gaussian_rho2"]).reshape(2, -1)) < TOL


def test_generic_full_model(dev):
    """Unrolled_ADMM(n=2, 'Gaussian') with SubNet + ResUNet (seed-1234 weights) at 45 x 60."""
    from gdeconv.weights import make_state_dict
    from models.Unrolled_ADMM import Unrolled_ADMM
    g = golden("sizes.npz")
    obs, psf, alpha = (T(g[k]).to(dev) for k in ("full_obs", "full_psf", "full_alpha"))
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    m = Unrolled_ADMM(n_iters=2, llh="Gaussian")
    m.load_state_dict(make_state_dict(m, 1234))
    m = m.to(dev).eval()
    with torch.no_grad():
        out = m(obs, psf, alpha).cpu()
    assert report("Unrolled_ADMM(2, Gaussian) full model 45x60", out, T(g["full_out"])) < TOL


def test_generic_gauss2x_identity(dev):
    """UnrolledADMMGaussian(n=4) with the identity denoiser at 40 x 40 (80 x 80 padded grid)."""
    from gdeconv.weights import make_state_dict
    from models.unrolled_admm_gaussian import UnrolledADMMGaussian
    g = golden("sizes.npz")
    obs, psf, alpha, rho = (T(g[k]) for k in ("gx_obs", "gx_psf", "gx_alpha", "gx_rho"))
    m = UnrolledADMMGaussian(n_iters=4)
    m.load_state_dict(make_state_dict(m, 1234))
    m.Z = torch.nn.Identity()
    m = m.to(dev).eval()
    with torch.no_grad():
        assert nerr(m.init(psf.to(dev), alpha.to(dev)).cpu().reshape(2, -1), rho.reshape(2, -1)) < TOL
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert report("UnrolledADMMGaussian(4) identity 40x40", out, T(g["gx_out"])) < TOL


def test_generic_gauss2x_backward(dev):
    """The X update's HIP backward on a generic 2x grid (side 42 -> 84 x 84): forward and gradients
    against autograd through the fp64 oracle (models/unrolled_admm_gaussian.py:89-93)."""
    from gdeconv import engine
    from gdeconv.synth import make_batch
    obs, psf, alpha, _ = make_batch(2, 42, h=42, seed=9, device=dev)
    st = engine.GaussXState(obs, psf, alpha)
    gen = torch.Generator().manual_seed(5)
    a, b, u = (torch.randn(obs.shape, generator=gen).to(dev) for _ in range(3))
    rho = torch.tensor([0.7, 1.3], device=dev).view(2, 1, 1, 1)
    z = a.clone().requires_grad_(True)
    r = rho.clone().requires_grad_(True)
    uu = u.clone().requires_grad_(True)
    x = engine.gx_x_update(st, z, uu, r)
    (x * b).sum().backward()
    _, Y, Ht, HtH = O.gx_spectra(obs.cpu().double(), psf.cpu().double())
    z64 = a.cpu().double().requires_grad_(True)
    u64 = u.cpu().double().requires_grad_(True)
    r64 = rho.cpu().double().requires_grad_(True)
    x64 = O.gx_x_update(Y, Ht, HtH, z64, u64, r64)
    assert nerr(x.detach().cpu(), x64.detach()) < TOL
    (x64 * b.cpu().double()).sum().backward()
    assert nerr(z.grad.cpu(), z64.grad) < TOL
    assert nerr(uu.grad.cpu(), u64.grad) < TOL
    assert float(((r.grad.cpu().double() - r64.grad).abs() / r64.grad.abs()).max()) < TOL


@pytest.mark.parametrize("H,W", [(40, 56), (48, 30)])
def test_generic_gauss2x_rect(dev, H, W):
    """UnrolledADMMGaussian(n=4) with the identity denoiser on a NON-SQUARE image (2H x 2W padded grid,
    pad_double per axis, models/unrolled_admm_gaussian.py:117-152): the SubNet's rhos, init_l2's z0 and
    the forward's output against the reference (tests/golden/make_golden_gx_rect.py)."""
    from gdeconv import engine
    from gdeconv.weights import make_state_dict
    from models.unrolled_admm_gaussian import UnrolledADMMGaussian
    g = golden("gauss2x_rect.npz")
    t = f"{H}x{W}"
    obs, psf, alpha = (T(g[f"{t}_{k}"]).to(dev) for k in ("obs", "psf", "alpha"))
    m = UnrolledADMMGaussian(n_iters=4)
    m.load_state_dict(make_state_dict(m, 1234))
    m.Z = torch.nn.Identity()
    m = m.to(dev).eval()
    with torch.no_grad():
        assert nerr(m.init(psf, alpha).cpu().reshape(2, -1), T(g[f"{t}_rho"]).reshape(2, -1)) < TOL
        st = engine.GaussXState(obs, psf, alpha)
        assert report(f"UnrolledADMMGaussian init_l2 {t}", st.init().cpu(), T(g[f"{t}_z0"])) < TOL
        out = m(obs, psf, alpha).cpu()
    assert report(f"UnrolledADMMGaussian(4) identity {t}", out, T(g[f"{t}_out"])) < TOL


def test_generic_gauss2x_rect_backward(dev):
    """The X update's HIP backward on a non-square 2x grid (30 x 44 -> 60 x 88) against autograd through
    the fp64 oracle."""
    from gdeconv import engine
    from gdeconv.synth import make_batch
    obs, _, alpha, _ = make_batch(2, 30, 44, h=30, seed=11, device=dev)
    gen = torch.Generator().manual_seed(6)
    psf = torch.rand(2, 1, 30, 44, generator=gen).to(dev)
    psf = psf / psf.sum(dim=(-2, -1), keepdim=True)
    st = engine.GaussXState(obs, psf, alpha)
    a, b, u = (torch.randn(obs.shape, generator=gen).to(dev) for _ in range(3))
    rho = torch.tensor([0.9, 1.6], device=dev).view(2, 1, 1, 1)
    z = a.clone().requires_grad_(True)
    r = rho.clone().requires_grad_(True)
    uu = u.clone().requires_grad_(True)
    x = engine.gx_x_update(st, z, uu, r)
    (x * b).sum().backward()
    _, Y, Ht, HtH = O.gx_spectra(obs.cpu().double(), psf.cpu().double())
    z64 = a.cpu().double().requires_grad_(True)
    u64 = u.cpu().double().requires_grad_(True)
    r64 = rho.cpu().double().requires_grad_(True)
    x64 = O.gx_x_update(Y, Ht, HtH, z64, u64, r64)
    assert nerr(x.detach().cpu(), x64.detach()) < TOL
    (x64 * b.cpu().double()).sum().backward()
    assert nerr(z.grad.cpu(), z64.grad) < TOL
    assert nerr(uu.grad.cpu(), u64.grad) < TOL
    assert float(((r.grad.cpu().double() - r64.grad).abs() / r64.grad.abs()).max()) < TOL


def test_generic_batch_invariance_and_odd_batch(dev):
    """Chunked pipeline over a ragged batch at a generic size: every galaxy equals its solo run."""
    from gdeconv import _lib, engine
    from gdeconv.synth import make_batch
    lib = _lib.load()
    N = 23
    obs, psf, alpha, _ = make_batch(N, 72, 88, h=32, seed=31, device=dev)
    old = lib.gd_set_chunk_bytes(1 << 20)  # force many chunks over the 2 pipeline streams
    try:
        full = engine.wiener(obs, psf, alpha).cpu()
        rl = engine.richardson_lucy(obs, psf, 3).cpu()
    finally:
        lib.gd_set_chunk_bytes(old)
    for i in (0, 11, N - 1):
        solo = engine.wiener(obs[i:i + 1], psf[i:i + 1], alpha[i:i + 1]).cpu()
        assert torch.equal(full[i:i + 1], solo)
        assert torch.equal(rl[i:i + 1], engine.richardson_lucy(obs[i:i + 1], psf[i:i + 1], 3).cpu())
    ref = O.wiener(obs[:2].cpu(), psf[:2].cpu(), alpha[:2].cpu())
    assert nerr(full[:2], ref) < TOL


@pytest.mark.parametrize("H,W", [(1638, 1536), (1200, 1400)])
def test_generic_large_images_admm_and_wiener(dev, H, W):
    """The largest images the runtime-planned path takes (1638 per side: a two-image workgroup's lines in
    64 KiB of LDS): Wiener and Unrolled_ADMM(2, Gaussian) with an identity denoiser against the fp64 oracle."""
    from gdeconv import engine
    from gdeconv.synth import make_batch
    obs, psf, alpha, _ = make_batch(1, H, W, h=48, seed=H + W)
    wien = engine.wiener(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert nerr(wien, O.wiener(obs.double(), psf.double(), alpha.double())) < TOL
    rho1 = torch.full((1, 1, 1, 2), 0.9)
    rho2 = torch.full((1, 1, 1, 2), 1.1)
    m = _spectral_model(2, "Gaussian", dev, rho1, rho2)
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    ref = O.admm_forward(obs.double(), psf.double(), alpha.double(), rho1.double(), rho2.double(), "Gaussian")
    e = nerr(out, ref)
    print(f"{H}x{W}: Wiener / ADMM(2) vs fp64 oracle, ADMM {e:.2e}")
    assert e < TOL


@pytest.mark.parametrize("H,W", [(4096, 4096), (2053, 2500)])
def test_generic_big_lines_wiener_rl_admm(dev, H, W):
    """Lines longer than 1638 points (up to 4096: the whole 160 KiB of a CU's LDS per workgroup, dynamic LDS above
    64 KiB allowed per kernel): Wiener, Richardson-Lucy(3) and Unrolled_ADMM(2, Gaussian) with an identity denoiser
    against the fp64 oracle; 2053 is prime (one odd-prime DFT stage of 2053 points)."""
    from gdeconv import engine
    from gdeconv.synth import make_batch
    # 2053 x 2500: two galaxies, so the chunked pipeline (one galaxy per 96 MiB chunk here) runs its two streams
    obs, psf, alpha, _ = make_batch(1 if H == 4096 else 2, H, W, h=48, seed=H + 3 * W)
    wien = engine.wiener(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    assert report(f"Wiener {H}x{W}", wien, O.wiener(obs.double(), psf.double(), alpha.double())) < TOL
    rl = engine.richardson_lucy(obs.to(dev), psf.to(dev), 3).cpu()
    assert report(f"Richardson-Lucy(3) {H}x{W}", rl, O.richardson_lucy(obs.double(), psf.double(), 3)) < TOL
    rho1 = torch.full((obs.shape[0], 1, 1, 2), 0.9)
    rho2 = torch.full((obs.shape[0], 1, 1, 2), 1.1)
    m = _spectral_model(2, "Gaussian", dev, rho1, rho2)
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    ref = O.admm_forward(obs.double(), psf.double(), alpha.double(), rho1.double(), rho2.double(), "Gaussian")
    assert report(f"Unrolled_ADMM(2) identity {H}x{W}", out, ref) < TOL
    if H != 4096:  # the Poisson chain (V step per pixel in the row-inverse kernel) at a prime side
        m = _spectral_model(2, "Poisson", dev, rho1, rho2)
        with torch.no_grad():
            out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
        ref = O.admm_forward(obs.double(), psf.double(), alpha.double(), rho1.double(), rho2.double(), "Poisson")
        assert report(f"Unrolled_ADMM(2, Poisson) identity {H}x{W}", out, ref) < TOL


def test_generic_gauss2x_big_grid(dev):
    """UnrolledADMMGaussian beyond round 5's 818 cap: 1024 x 1024 images on the 2048 x 2048 padded grid (lines longer
    than 1638 points), init_l2 and one X update against the fp64 oracle (models/unrolled_admm_gaussian.py:89-93)."""
    from gdeconv import engine
    from gdeconv.synth import make_batch
    obs, psf, alpha, _ = make_batch(1, 1024, h=1024, seed=21, device=dev)
    st = engine.GaussXState(obs, psf, alpha)
    _, Y, Ht, HtH = O.gx_spectra(obs.cpu().double(), psf.cpu().double())
    z0 = st.init().cpu()
    assert report("UnrolledADMMGaussian init_l2 1024x1024", z0, O.gx_init_l2(Y, Ht, HtH, alpha.cpu().double())) < TOL
    gen = torch.Generator().manual_seed(3)
    z, u = (torch.randn(obs.shape, generator=gen) for _ in range(2))
    rho = torch.tensor([0.8]).view(1, 1, 1, 1)
    x = engine.gx_x_update(st, z.to(dev), u.to(dev), rho.to(dev)).cpu()
    ref = O.gx_x_update(Y, Ht, HtH, z.double(), u.double(), rho.double())
    assert report("UnrolledADMMGaussian X update 1024x1024", x, ref) < TOL


@pytest.mark.parametrize("L,llh", [(48, "Poisson"), (80, "Poisson"), (80, "Gaussian"), (144, "Gaussian")])
def test_fused_one_workgroup_kernels_shared_psf_and_scalar_alpha(dev, L, llh):
    """The fused one-workgroup kernels (k_pois_small*, k_gal_mid*) with ONE PSF for the whole batch (psf batch 1:
    galaxy stride 0) and a Python-number alpha (stride 0), against the chains and the fp64 oracle."""
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    lib = _lib.load()
    N, n = 3, 2
    obs, psf, alpha, _ = make_batch(N, L, h=32, seed=7 + L, device=dev)
    psf1 = psf[:1].contiguous()
    rho1 = torch.tensor([0.8, 1.3]).float()
    rho2 = torch.tensor([1.1, 0.6]).float()
    m = _spectral_model(n, llh, dev, rho1.to(dev), rho2.to(dev))
    with torch.no_grad():
        out_f = m(obs, psf1, 0.7).cpu()
        old, old_i = lib.gd_set_fused_iteration(0), lib.gd_set_fused_init(0)
        try:
            out_c = m(obs, psf1, 0.7).cpu()
        finally:
            lib.gd_set_fused_iteration(old)
            lib.gd_set_fused_init(old_i)
    a64 = torch.full((N, 1, 1, 1), 0.7, dtype=torch.float64)
    ref = O.admm_forward(obs.cpu().double(), psf1.cpu().double().expand(N, 1, 32, 32), a64,
                         rho1.double().view(1, 1, 1, n).expand(N, 1, 1, n), rho2.double().view(1, 1, 1, n).expand(N, 1, 1, n), llh)
    e_fc, e_f = nerr(out_f, out_c), nerr(out_f, ref)
    print(f"{llh} {L}^2 shared PSF, scalar alpha: fused vs chain {e_fc:.2e}, vs fp64 oracle {e_f:.2e}")
    assert e_fc < 5e-6 and e_f < TOL


@pytest.mark.parametrize("L", [32, 48, 64, 80, 96, 112])
@pytest.mark.parametrize("n", [0, 1, 3])
def test_fused_poisson_small_matches_chain_and_oracle(dev, L, n):
    """Poisson (the reference's default llh) at L <= 112: the init (k_pois_small_init: init_l2 and the first V
    step) and each iteration (k_pois_small) in one launch, both images' packed row spectra in LDS, against the
    chains (gd_set_fused_iteration(0), gd_set_fused_init(0)) and the fp64 oracle: x0 alone (n = 0), last-only
    (n = 1) and middle + last iterations, ragged batch of 5."""
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    lib = _lib.load()
    N = 5
    obs, psf, alpha, _ = make_batch(N, L, h=min(48, L // 2 * 2 - 16 if L < 64 else 48), seed=61 + n + L, device=dev)
    gen = torch.Generator().manual_seed(91 + n + L)
    rho1 = (0.5 + torch.rand(N, 1, 1, n, generator=gen)).float()
    rho2 = (0.5 + torch.rand(N, 1, 1, n, generator=gen)).float()
    m = _spectral_model(n, "Poisson", dev, rho1, rho2)
    with torch.no_grad():
        out_f = m(obs, psf, alpha).cpu()
        old, old_i = lib.gd_set_fused_iteration(0), lib.gd_set_fused_init(0)
        try:
            out_c = m(obs, psf, alpha).cpu()
        finally:
            lib.gd_set_fused_iteration(old)
            lib.gd_set_fused_init(old_i)
    ref = O.admm_forward(obs.cpu().double(), psf.cpu().double(), alpha.cpu().double(), rho1.double(), rho2.double(),
                         "Poisson")
    e_fc, e_f, e_c = nerr(out_f, out_c), nerr(out_f, ref), nerr(out_c, ref)
    print(f"Poisson {L}^2 n={n}: fused vs chain {e_fc:.2e}, vs fp64 oracle {e_f:.2e} (chain {e_c:.2e})")
    assert e_fc < 5e-6
    assert e_f < TOL


@pytest.mark.parametrize("L", [64, 80, 96, 112, 128, 144, 160])
@pytest.mark.parametrize("n", [0, 1, 2, 4])
def test_generic_fused_mid_matches_chain_and_oracle(dev, L, n):
    """64^2 ... 160^2 Gaussian iterations in one launch per iteration (k_gal_mid: the half spectrum
    in LDS, 16-lane x L/16-point line transforms with radix 5, 7, 9, 10) and the init in one launch
    (k_gal_mid_init) against the runtime-planned chains (gd_set_fused_iteration(0), gd_set_fused_init(0)) and the
    fp64-capable oracle: n = 0 is init_l2 alone (x0), then first / middle / last / first-and-last iterations,
    ragged batch of 5."""
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    lib = _lib.load()
    N = 5
    obs, psf, alpha, _ = make_batch(N, L, h=48, seed=41 + n + L, device=dev)
    gen = torch.Generator().manual_seed(77 + n)
    rho1 = (0.5 + torch.rand(N, 1, 1, n, generator=gen)).float()
    rho2 = (0.5 + torch.rand(N, 1, 1, n, generator=gen)).float()
    m = _spectral_model(n, "Gaussian", dev, rho1, rho2)
    with torch.no_grad():
        out_f = m(obs, psf, alpha).cpu()
        old, old_i = lib.gd_set_fused_iteration(0), lib.gd_set_fused_init(0)
        try:
            out_c = m(obs, psf, alpha).cpu()
        finally:
            lib.gd_set_fused_iteration(old)
            lib.gd_set_fused_init(old_i)
    ref = O.admm_forward(obs.cpu().double(), psf.cpu().double(), alpha.cpu().double(), rho1.double(), rho2.double(),
                         "Gaussian")
    e_fc, e_f, e_c = nerr(out_f, out_c), nerr(out_f, ref), nerr(out_c, ref)
    print(f"{L}^2 n={n}: fused vs chain {e_fc:.2e}, vs fp64 oracle {e_f:.2e} (chain {e_c:.2e})")
    assert e_fc < 5e-6
    assert e_f < TOL and e_c < TOL

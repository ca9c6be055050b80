"""Per-pixel parity against fp64: the engine is no worse than the reference (north_star's "1e-5 rel
fp32 per pixel" clause).

A second correct fp32 FFT cannot meet 1e-5 per pixel against the first one: the reference's own fp32
output sits up to 2.9e-3 (Wiener) and 1.2e-1 (Tikhonov-Laplacian, 192 x 160) per pixel away from the
exact result, because a deconvolution amplifies rounding where |H|^2 is small.  So every spectral-only
golden case here is measured three ways on the same inputs:

  engine (GPU, fp32)   vs  the fp64 oracle (oracle/admm_oracle.py in double)
  reference (golden)   vs  the fp64 oracle
  engine               vs  reference

with both the normwise metric (the gate, <= 1e-5) and the floored per-pixel metric (its max, its median
and 99th percentile over all pixels, and its 32nd-largest value).  The bar: engine-vs-fp64 <= 2 x
reference-vs-fp64 at the 99th percentile and at the 32nd-largest pixel of the floored per-pixel error,
i.e. the engine's fp32 arithmetic is within a factor of two of the reference's own over the tail of the
per-pixel error distribution.

The MAX of the floored per-pixel error is recorded but not bounded: it is set by the one pixel nearest a
zero crossing of the output, so between two equally accurate fp32 implementations its ratio is the ratio
of two random rounding draws at that pixel.  The reference against itself shows it: its own rfft2 path
vs its fftn path scatters to 2.4x on the max while staying <= 2x at p99 / the 32nd-largest pixel
(tests/test_oracle_golden.py::test_pixel_max_is_noise_between_two_reference_fft_paths).
Every case is appended to $GD_PARITY_LOG (JSON lines) when set.
"""
import json
import os

import numpy as np
import pytest
import torch

import admm_oracle as O
from conftest import golden, parity_gate

pytestmark = pytest.mark.gpu

TOL = 1e-5
BOUND = 2.0
F64 = torch.float64
SIZES = [(40, 40), (64, 48), (45, 60), (97, 80), (192, 160), (45, 61), (255, 255)]


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))



def _nerr(a, b):
    return float(O.normwise_error(a, b).max())


def _pix(a, b):
    return float(O.pixel_error_floored(a, b).max())


def pix_quantiles(a, ref, k_tail=32):
    """[median, 99th percentile, k_tail-th largest] over all pixels of the floored per-pixel relative
    error (the metric of O.pixel_error_floored before its max).  The tail point is the 32nd-largest
    pixel (p99.9 at 256^2, p99.3 for two 48^2 galaxies): far enough from the max to be a statistic of
    the error distribution rather than one pixel's rounding draw."""
    a = a.detach().double().cpu().reshape(a.shape[0], -1)
    ref = ref.detach().double().cpu().reshape(ref.shape[0], -1)
    den = torch.maximum(ref.abs(), 1e-5 * ref.abs().amax(1, keepdim=True)).clamp_min(1e-300)
    r = ((a - ref).abs() / den).flatten()
    tail = float(torch.topk(r, min(k_tail, r.numel())).values[-1])
    return [float(torch.quantile(r, 0.5)), float(torch.quantile(r, 0.99)), tail]


def check(tag, out, gold, ref64):
    """Record both columns for one case and apply the bar; returns the record."""
    qe, qr = pix_quantiles(out, ref64), pix_quantiles(gold, ref64)
    rec = {"case": tag,
           "engine_vs_fp64_pixel_p50_p99_top32": qe, "reference_vs_fp64_pixel_p50_p99_top32": qr,
           "engine_vs_fp64_normwise": _nerr(out, ref64), "engine_vs_fp64_per_pixel": _pix(out, ref64),
           "reference_vs_fp64_normwise": _nerr(gold, ref64), "reference_vs_fp64_per_pixel": _pix(gold, ref64),
           "engine_vs_reference_normwise": _nerr(out, gold), "engine_vs_reference_per_pixel": _pix(out, gold)}
    rec["per_pixel_ratio"] = rec["engine_vs_fp64_per_pixel"] / max(rec["reference_vs_fp64_per_pixel"], 1e-300)
    print("[pixel-parity] " + " ".join(f"{k}={v:.3e}" if isinstance(v, float) else f"{k}={v}" for k, v in rec.items()))
    if os.environ.get("GD_PARITY_DUMP"):   # raw outputs for offline analysis
        d = os.environ["GD_PARITY_DUMP"]
        os.makedirs(d, exist_ok=True)
        name = "".join(c if c.isalnum() else "_" for c in tag)[:80]
        np.savez_compressed(os.path.join(d, name + ".npz"), out=out.numpy(), gold=gold.numpy(), ref64=ref64.numpy())
    log = os.environ.get("GD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(rec) + "\n")
    # the normwise gate, per galaxy (conftest.parity_gate): engine vs fp64 <= 1e-5 and engine vs the
    # reference <= 1e-5, relaxed only for the listed ill-conditioned cases
    rec["gate"] = parity_gate(tag, out, gold, ref64, tol=TOL)
    for i in (1, 2):   # p99, 32nd-largest
        assert qe[i] <= BOUND * qr[i], rec
    return rec


def _spectral_model(n, llh, dev, rho1, rho2):
    from models.Unrolled_ADMM import Unrolled_ADMM
    m = Unrolled_ADMM(n_iters=n, llh=llh).to(dev).eval()
    m.Z = torch.nn.Identity()
    m.rhos = lambda k, a: (rho1.to(dev), rho2.to(dev))
    return m


# ------------------------------------------------------------------ compile-time-planned sizes
@pytest.mark.parametrize("tag", ["48", "256"])
@pytest.mark.parametrize("conj", [False, True])
def test_conv(dev, tag, conj):
    from gdeconv import engine
    g = golden("otf_conv.npz")
    obs, psf = T(g[f"obs{tag}"]), T(g[f"psf{tag}"])
    L = obs.shape[-1]
    out = engine.conv_half(engine.psf_to_otf_half(psf.to(dev), 1, L, L), obs.to(dev), conj=conj).cpu()
    _, H = O.psf_to_otf(psf.double(), obs.size(), dtype=F64)
    ref64 = O.conv_fft_batch(torch.conj(H) if conj else H, obs.double())
    check(f"conv_fft_batch{'(conj H)' if conj else ''} {tag}^2", out, T(g[f"conv_{'Ht' if conj else 'H'}{tag}"]), ref64)


@pytest.mark.parametrize("tag", ["48", "256"])
def test_wiener(dev, tag):
    from models.Wiener import Wiener
    g = golden("wiener_rl.npz")
    o, p, a = (T(g[k + tag]) for k in ("obs", "psf", "alpha"))
    out = Wiener()(o.to(dev), p.to(dev), a.to(dev)).cpu()
    check(f"Wiener {tag}^2", out, T(g[f"wiener{tag}"]), O.wiener(o.double(), p.double(), a.double()))


@pytest.mark.parametrize("tag", ["48", "256"])
@pytest.mark.parametrize("n", [10, 100])
def test_richardson_lucy(dev, tag, n):
    from models.Richard_Lucy import Richard_Lucy
    g = golden("wiener_rl.npz")
    o, p = T(g["obs" + tag]), T(g["psf" + tag])
    out = Richard_Lucy(n)(o.to(dev), p.to(dev)).cpu()
    check(f"Richard_Lucy({n}) {tag}^2", out, T(g[f"rl{n}_{tag}"]), O.richardson_lucy(o.double(), p.double(), n))


@pytest.mark.parametrize("tag", ["48", "256"])
@pytest.mark.parametrize("filt", ["Identity", "Laplacian"])
@pytest.mark.parametrize("lam", [1.0, 0.37])
def test_tikhonov(dev, tag, filt, lam):
    from gdeconv.models import Tikhonov
    g = golden("tikhonov.npz")
    obs, psf, alpha = (T(g[k + tag]) for k in ("obs", "psf", "alpha"))
    yp = torch.clamp_min(obs, 0)
    out = Tikhonov(filter=filt)(yp.to(dev), psf.to(dev), alpha.to(dev), torch.tensor(lam)).cpu()
    ref64 = O.tikhonov(yp.double(), psf.double(), alpha.double(), torch.tensor(lam, dtype=F64), filt)
    check(f"Tikhonov({filt}, lam={lam}) {tag}^2", out, T(g[f"tik_{filt}_{lam}_{tag}"]), ref64)


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
def test_admm256_identity(dev, llh):
    """configs[2]'s path: Unrolled_ADMM(n=8) spectral engine (identity denoiser) at 256^2."""
    g = golden("admm256_id.npz")
    obs, psf, alpha = T(g["obs"]), T(g["psf"]), T(g["alpha"])
    r1, r2 = T(g[f"{llh}_rho1"]), T(g[f"{llh}_rho2"])
    with torch.no_grad():
        out = _spectral_model(8, llh, dev, r1, r2)(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    ref64 = O.admm_forward(obs.double(), psf.double(), alpha.double(), r1.double(), r2.double(), llh)
    check(f"Unrolled_ADMM(8, {llh}) identity 256^2", out, T(g[f"{llh}_out"]), ref64)


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
@pytest.mark.parametrize("n", [2, 8])
def test_admm48_replay(dev, llh, n):
    """Unrolled_ADMM at 48^2 (configs[0]/[1] stamp) with the reference's own per-iteration denoiser
    outputs fed back in: every spectral step of the loop, both llh."""
    g = golden("admm48.npz")
    if f"{llh}_n{n}_z" not in g.files:
        pytest.skip("no per-iteration trace in the fixture")
    obs, psf, alpha = T(g["obs"]), T(g["psf"]), T(g["alpha"])
    zs = T(g[f"{llh}_n{n}_z"])
    r1, r2 = T(g[f"{llh}_n{n}_rho1"]), T(g[f"{llh}_n{n}_rho2"])
    seen = []

    class Replay(torch.nn.Module):
        def forward(self, zin):
            seen.append(1)
            return zs[len(seen) - 1].to(zin.device)

    m = _spectral_model(n, llh, dev, r1, r2)
    m.Z = Replay()
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    it = iter(range(n))
    ref64 = O.admm_forward(obs.double(), psf.double(), alpha.double(), r1.double(), r2.double(), llh,
                           denoise=lambda t: zs[next(it)].double())
    check(f"Unrolled_ADMM({n}, {llh}) 48^2, reference denoiser outputs replayed", out, T(g[f"{llh}_n{n}_out"]), ref64)


# ------------------------------------------------------------------ runtime-planned sizes
def _load(H, W):
    g = golden("sizes.npz")
    t = f"{H}x{W}"
    return g, t, T(g[f"{t}_obs"]), T(g[f"{t}_psf"]), T(g[f"{t}_alpha"])


@pytest.mark.parametrize("H,W", SIZES)
def test_generic_spectral_ops(dev, H, W):
    from gdeconv import engine
    from gdeconv.models import Tikhonov
    from models.Richard_Lucy import Richard_Lucy
    from models.Wiener import Wiener
    g, t, obs, psf, alpha = _load(H, W)
    o, p, a = obs.to(dev), psf.to(dev), alpha.to(dev)
    od, pd, ad = obs.double(), psf.double(), alpha.double()
    _, Hd = O.psf_to_otf(pd, obs.size(), dtype=F64)
    otf = engine.psf_to_otf_half(p, obs.shape[0], H, W)
    check(f"conv_fft_batch {t}", engine.conv_half(otf, o).cpu(), T(g[f"{t}_conv_H"]), O.conv_fft_batch(Hd, od))
    check(f"conv_fft_batch(conj H) {t}", engine.conv_half(otf, o, conj=True).cpu(), T(g[f"{t}_conv_Ht"]),
          O.conv_fft_batch(torch.conj(Hd), od))
    check(f"Wiener {t}", Wiener()(o, p, a).cpu(), T(g[f"{t}_wiener"]), O.wiener(od, pd, ad))
    check(f"Richard_Lucy(10) {t}", Richard_Lucy(10)(o, p).cpu(), T(g[f"{t}_rl10"]), O.richardson_lucy(od, pd, 10))
    yp = torch.clamp_min(obs, 0)
    for filt in ("Identity", "Laplacian"):
        out = Tikhonov(filter=filt)(yp.to(dev), p, a, torch.tensor(0.37)).cpu()
        check(f"Tikhonov({filt}) {t}", out, T(g[f"{t}_tik_{filt}"]),
              O.tikhonov(yp.double(), pd, ad, torch.tensor(0.37, dtype=F64), filt))


@pytest.mark.parametrize("H,W", [(255, 255), (192, 160)])
def test_generic_tikhonov_second_lambdas(dev, H, W):
    from gdeconv.models import Tikhonov
    g = golden("tik_sizes.npz")
    t = f"{H}x{W}"
    obs, psf, alpha = (T(g[f"{t}_{k}"]) for k in ("obs", "psf", "alpha"))
    yp = torch.clamp_min(obs, 0)
    for lam in (0.05, 2.0):   # make_golden_tik.LAMS
        for filt in ("Identity", "Laplacian"):
            out = Tikhonov(filter=filt)(yp.to(dev), psf.to(dev), alpha.to(dev), torch.tensor(lam)).cpu()
            check(f"Tikhonov({filt}, lam={lam}) {t}", out, T(g[f"{t}_tik_{filt}_{lam}"]),
                  O.tikhonov(yp.double(), psf.double(), alpha.double(), torch.tensor(lam, dtype=F64), filt))


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
@pytest.mark.parametrize("H,W", SIZES)
def test_generic_admm_identity(dev, H, W, llh):
    g, t, obs, psf, alpha = _load(H, W)
    r1, r2 = T(g[f"{t}_{llh}_rho1"]), T(g[f"{t}_{llh}_rho2"])
    with torch.no_grad():
        out = _spectral_model(4, llh, dev, r1, r2)(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    ref64 = O.admm_forward(obs.double(), psf.double(), alpha.double(), r1.double(), r2.double(), llh)
    check(f"Unrolled_ADMM(4, {llh}) identity {t}", out, T(g[f"{t}_{llh}_out"]), ref64)


def test_gauss2x_identity(dev):
    """UnrolledADMMGaussian(4) identity denoiser at 40 x 40 (80 x 80 padded grid), the reference's rhos."""
    from gdeconv.weights import make_state_dict
    from models.unrolled_admm_gaussian import UnrolledADMMGaussian
    g = golden("sizes.npz")
    obs, psf, alpha, rho = (T(g[k]) for k in ("gx_obs", "gx_psf", "gx_alpha", "gx_rho"))
    m = UnrolledADMMGaussian(n_iters=4)
    m.load_state_dict(make_state_dict(m, 1234))
    m.Z = torch.nn.Identity()
    m = m.to(dev).eval()
    m.__dict__["init"] = lambda k, a: rho.to(dev)   # the reference's rhos (instance attribute shadows the SubNet)
    with torch.no_grad():
        out = m(obs.to(dev), psf.to(dev), alpha.to(dev)).cpu()
    ref64 = O.gx_forward(obs.double(), psf.double(), alpha.double(), rho.double())
    check("UnrolledADMMGaussian(4) identity 40x40", out, T(g["gx_out"]), ref64)

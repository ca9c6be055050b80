"""Seeded synthetic galaxy batches; there is no network for the reference's
GalSim/COSMOS dataset (``generate_data.py:114-333``), so inputs follow its recipe analytically:

* gt  : elliptical exponential profile, centre offset U(-1,1) px, half-light radius U(2,6)*(H/48) px,
        ellipticity U(0,0.3), position angle U(0,pi);
* psf : h x h (h even, default 48) Moffat(beta=3.5) or Gaussian with FWHM U(3,5) px, centred on
        pixel (h/2, h/2), normalised to sum 1/16 (the 4x4 average down-sample of
        ``generate_data.py:251``, same as ``tutorials/psf.pth``);
* obs : circular conv(psf, gt) + N(0, sigma^2), sigma = 19.04 ADU (``generate_data.py:195-202``),
        gt flux scaled so that SNR = ||conv(psf, gt)||_2 / sigma ~ U(20, 200) (``:241-243``);
* alpha = per-galaxy obs mean, [N,1,1,1] (``utils/utils_data.py:100-101``).

Parameters are drawn on the CPU from ``torch.Generator().manual_seed(seed)``; images are built on
``device`` (the bench builds N=4096 256^2 batches directly in HBM).
"""
import math

import torch

SIGMA_NOISE = 19.04


def _psf_shift_to_origin(psf, H, W):
    """Zero-pad the h x h PSF to H x W and roll pixel (h/2, h/2) to (0, 0)."""
    N, _, h, w = psf.shape
    big = torch.zeros(N, 1, H, W, dtype=psf.dtype, device=psf.device)
    big[:, :, :h, :w] = psf
    return torch.roll(big, shifts=(-(h // 2), -(w // 2)), dims=(2, 3))


def make_batch(N, H, W=None, h=48, seed=20250307, device="cpu", dtype=torch.float32):
    """Return (obs [N,1,H,W], psf [N,1,h,h], alpha [N,1,1,1], gt [N,1,H,W])."""
    W = H if W is None else W
    if h > min(H, W) or h % 2:
        raise ValueError("psf side must be even and <= the image side")
    g = torch.Generator().manual_seed(seed)
    u = lambda lo, hi: lo + (hi - lo) * torch.rand(N, generator=g, dtype=torch.float64)  # noqa
    cx, cy = u(-1, 1), u(-1, 1)
    hlr = u(2, 6) * (H / 48.0)
    ell = u(0, 0.3)
    theta = u(0, math.pi)
    fwhm = u(3, 5)
    moffat = torch.rand(N, generator=g) < 0.5
    snr = u(20, 200)
    noise = torch.randn(N, 1, H, W, generator=g, dtype=torch.float32)

    dev = torch.device(device)
    f64 = torch.float64
    col = lambda t: t.to(dev, f64).view(N, 1, 1, 1)  # noqa: E731
    yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=f64),
                            torch.arange(W, device=dev, dtype=f64), indexing="ij")
    dx = xx[None, None] - (W / 2 + col(cx))
    dy = yy[None, None] - (H / 2 + col(cy))
    ct, st = torch.cos(col(theta)), torch.sin(col(theta))
    q = (1 - col(ell)) / (1 + col(ell))                     # axis ratio from ellipticity
    xr, yr = dx * ct + dy * st, -dx * st + dy * ct
    r = torch.sqrt(xr ** 2 * q + yr ** 2 / q)
    rs = col(hlr) / 1.678                                    # exponential: r_half = 1.678 r_s
    gt = torch.exp(-r / rs)

    py, px = torch.meshgrid(torch.arange(h, device=dev, dtype=f64),
                            torch.arange(h, device=dev, dtype=f64), indexing="ij")
    pr2 = (px[None, None] - h // 2) ** 2 + (py[None, None] - h // 2) ** 2
    fw = col(fwhm)
    beta = 3.5
    alpha_m = fw / (2 * torch.sqrt(torch.tensor(2.0 ** (1 / beta) - 1, dtype=f64)))
    mof = (1 + pr2 / alpha_m ** 2) ** (-beta)
    gau = torch.exp(-pr2 / (2 * (fw / 2.3548200450309493) ** 2))
    psf = torch.where(moffat.to(dev).view(N, 1, 1, 1), mof, gau)
    psf = psf / psf.sum(dim=(2, 3), keepdim=True) / 16.0

    otf = torch.fft.rfft2(_psf_shift_to_origin(psf, H, W))
    clean = torch.fft.irfft2(torch.fft.rfft2(gt) * otf, s=(H, W))
    scale = col(snr) * SIGMA_NOISE / clean.flatten(1).norm(dim=1).view(N, 1, 1, 1)
    gt = gt * scale
    obs = clean * scale + SIGMA_NOISE * noise.to(dev, f64)
    alpha = obs.flatten(1).mean(1).view(N, 1, 1, 1)
    return obs.to(dtype), psf.to(dtype), alpha.to(dtype), gt.to(dtype)


__all__ = ["make_batch", "SIGMA_NOISE"]

"""ORACLE - TEST INFRASTRUCTURE ONLY.

CPU restatement (PyTorch CPU, fp32 by default, fp64 on request) of the reference's spectral
deconvolution math, op-for-op in the reference's order.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only
as the checker / the timed CPU baseline - the product path (``galaxy-deconv_amd/gdeconv``) never
imports it and fails loudly when its HIP library is missing.

Pinning: every function here is checked bit-for-bit (fp32) against golden vectors produced by
importing the reference itself read-only in the build container (``tests/golden/make_golden.py``
-> ``tests/golden/*.npz``; test ``tests/test_oracle_golden.py``).

Reference call sites followed (paths relative to the reference root):
  psf_to_otf          utils/utils_torch.py:79-92
  conv_fft_batch      utils/utils_torch.py:46-50  (fftn/ifftn over dims [2,3], :22-27)
  x_update            models/Unrolled_ADMM.py:315-319  (the *runtime* X_Update: the second class
                      definition shadows :93-101, so lhs = rho1*|H|^2 + rho2)
  v_update_poisson    models/Unrolled_ADMM.py:326-328
  v_update_gaussian   models/Unrolled_ADMM.py:335-336
  init_l2             models/Unrolled_ADMM.py:170-175
  admm_forward        models/Unrolled_ADMM.py:177-215
  wiener              models/Wiener.py:10-20
  richardson_lucy     models/Richard_Lucy.py:10-24
  tikhonov            models/Tikhonet.py:15-31 (+ laplacian_kernel, utils/utils_torch.py:95-99)
  gx_*                models/unrolled_admm_gaussian.py:85-152 (UnrolledADMMGaussian; pad_double /
                      crop_half utils/utils_torch.py:11-18)
"""
import torch

fftn = lambda x: torch.fft.fftn(x, dim=[2, 3])     # noqa: E731  utils/utils_torch.py:22-24
ifftn = lambda x: torch.fft.ifftn(x, dim=[2, 3])   # noqa: E731  utils/utils_torch.py:26-27


def psf_to_otf(ker, size, dtype=torch.float32):
    """utils/utils_torch.py:79-92: quadrant circular shift of the PSF into a zero image of
    ``size`` (PSF pixel (h/2, w/2) -> (0, 0)), then a full complex FFT over dims [2, 3]."""
    psf = torch.zeros(size, dtype=dtype)
    c = (ker.shape[2] + 1) // 2
    psf[:, :, :c, :c] = ker[:, :, c:, c:]
    psf[:, :, :c, -c:] = ker[:, :, c:, :c]
    psf[:, :, -c:, :c] = ker[:, :, :c, c:]
    psf[:, :, -c:, -c:] = ker[:, :, :c, :c]
    otf = torch.fft.fftn(psf, dim=[2, 3])
    return psf, otf


def conv_fft_batch(H, x):
    """utils/utils_torch.py:46-50: Re IFFT2(FFT2(x) * H)."""
    return ifftn(fftn(x) * H).real


def x_update(x0, x1, HtH, rho1, rho2):
    """models/Unrolled_ADMM.py:315-319 (runtime X_Update)."""
    lhs = rho1 * HtH + rho2
    rhs = fftn(rho1 * x0 + rho2 * x1)
    return ifftn(rhs / lhs).real


def v_update_poisson(v_tilde, y, rho2, alpha):
    """models/Unrolled_ADMM.py:326-328."""
    t1 = rho2 * v_tilde - alpha
    return 0.5 * (1 / rho2) * (-t1 + torch.sqrt(t1 ** 2 + 4 * y * rho2))


def v_update_gaussian(v_tilde, y, rho2):
    """models/Unrolled_ADMM.py:335-336."""
    return (rho2 * v_tilde + y) / (1 + rho2)


def init_l2(y, H, alpha):
    """models/Unrolled_ADMM.py:170-175: Wiener-style initialisation, clamped to [0, 1]."""
    Ht, HtH = torch.conj(H), torch.abs(H) ** 2
    rhs = fftn(conv_fft_batch(Ht, y / alpha))
    lhs = HtH + (1 / alpha)
    x0 = ifftn(rhs / lhs).real
    return torch.clamp(x0, 0, 1)


def admm_forward(y, kernel, alpha, rho1_iters, rho2_iters, llh="Gaussian", denoise=None,
                 trace=None):
    """models/Unrolled_ADMM.py:177-215 with the SubNet output given.

    ``rho1_iters``/``rho2_iters``: [N,1,1,n] (SubNet output, :188) or [n] (subnet=False, :204).
    ``denoise``: the Z step (callable on [N,1,H,W]); ``None`` = identity (spectral engine only).
    ``trace``: optional dict that receives per-iteration lists of v, z, x, u1, u2 (x includes x0).
    """
    N = y.shape[0]
    n_iters = rho1_iters.shape[-1]
    denoise = denoise if denoise is not None else (lambda t: t)
    y = torch.max(y, torch.zeros_like(y))
    _, H = psf_to_otf(kernel, y.size(), dtype=y.dtype)
    Ht, HtH = torch.conj(H), torch.abs(H) ** 2
    x = init_l2(y, H, alpha)
    u1 = torch.zeros_like(x)
    u2 = torch.zeros_like(y)
    if trace is not None:
        for k in ("v", "z", "x", "u1", "u2"):
            trace[k] = []
        trace["x"].append(x)
    for n in range(n_iters):
        if rho1_iters.dim() == 4:
            rho1 = rho1_iters[:, :, :, n].view(N, 1, 1, 1)
            rho2 = rho2_iters[:, :, :, n].view(N, 1, 1, 1)
        else:
            rho1, rho2 = rho1_iters[n], rho2_iters[n]
        if llh == "Poisson":
            v = v_update_poisson(conv_fft_batch(H, x) + u2, y, rho2, alpha)
        else:
            v = v_update_gaussian(conv_fft_batch(H, x) + u2, y / alpha, rho2)
        z = denoise(x + u1)
        x = x_update(z - u1, conv_fft_batch(Ht, v - u2), HtH, rho1, rho2)
        u1 = u1 + x - z
        u2 = u2 + conv_fft_batch(H, x) - v
        if trace is not None:
            for k, t in (("v", v), ("z", z), ("x", x), ("u1", u1), ("u2", u2)):
                trace[k].append(t)
    return x * alpha if llh == "Poisson" else x


def wiener(y, psf, alpha):
    """models/Wiener.py:10-20."""
    _, H = psf_to_otf(psf, y.size(), dtype=y.dtype)
    Ht, HtH = torch.conj(H), torch.abs(H) ** 2
    numerator = Ht * torch.fft.fftn(y, dim=[2, 3])
    divisor = HtH + 350 / alpha
    return torch.real(torch.fft.ifftn(numerator / divisor, dim=[2, 3]))


def richardson_lucy(y, psf, n_iters):
    """models/Richard_Lucy.py:10-24 (device handling dropped: CPU only)."""
    y = torch.max(y, torch.zeros_like(y))
    ones = torch.ones_like(y)
    _, H = psf_to_otf(psf, y.size(), dtype=y.dtype)
    Ht = torch.conj(H)
    x = y.clone()
    for _ in range(n_iters):
        Hx = conv_fft_batch(H, x)
        numerator = conv_fft_batch(Ht, y / Hx)
        divisor = conv_fft_batch(Ht, ones)
        x = x * numerator / divisor
    return x


def laplacian_kernel():
    """utils/utils_torch.py:95-99."""
    return torch.tensor([[[[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]]]])


def tikhonov(y, psf, alpha, lam, filt="Identity"):
    """models/Tikhonet.py:15-31 (Tikhonov.forward; y taken as given - Tikhonet applies max(y,0)).
    The Laplacian goes through psf_to_otf exactly as the reference's (odd 3x3: broadcast quadrants)."""
    _, H = psf_to_otf(psf, y.size(), dtype=y.dtype)
    Ht, HtH = torch.conj(H), torch.abs(H) ** 2
    numerator = Ht * torch.fft.fftn(y / alpha, dim=[2, 3])
    if filt == "Identity":
        divisor = HtH + lam
    else:
        _, Lf = psf_to_otf(laplacian_kernel().to(y.dtype), y.size(), dtype=y.dtype)
        divisor = HtH + lam * torch.abs(Lf) ** 2
    return torch.real(torch.fft.ifftn(numerator / divisor, dim=[2, 3]))


def pad_double(img):
    """utils/utils_torch.py:11-13."""
    H, W = img.shape[-2], img.shape[-1]
    return torch.nn.functional.pad(img, (W // 2, W // 2, H // 2, H // 2))


def crop_half(img):
    """utils/utils_torch.py:16-18."""
    H, W = img.shape[-2], img.shape[-1]
    return img[:, :, H // 4:3 * H // 4, W // 4:3 * W // 4]


def gx_spectra(y, kernel):
    """models/unrolled_admm_gaussian.py:118-123: max(y,0), Y, H, Ht, HtH on the 2x padded grid."""
    fs = torch.fft
    y = torch.maximum(y, torch.zeros_like(y))
    Y = fs.fft2(fs.ifftshift(pad_double(y), dim=(-2, -1)))
    H = fs.fft2(fs.ifftshift(pad_double(kernel), dim=(-2, -1)))
    return y, Y, torch.conj(H), torch.abs(H) ** 2


def gx_init_l2(Y, Ht, HtH, alpha):
    """models/unrolled_admm_gaussian.py:111-115."""
    rhs = Y * Ht
    lhs = HtH + (1 / alpha)
    x0 = torch.fft.fftshift(torch.fft.ifft2(rhs / lhs), dim=(-2, -1)).real
    return crop_half(x0)


def gx_x_update(Y, Ht, HtH, z, u, rho):
    """models/unrolled_admm_gaussian.py:89-93 (XUpdateGaussian.forward)."""
    fs = torch.fft
    lhs = rho + HtH
    rhs = Ht * Y + fs.fft2(fs.ifftshift(pad_double(rho * z - u), dim=(-2, -1)))
    x = fs.fftshift(fs.ifft2(rhs / lhs), dim=(-2, -1)).real
    return crop_half(x)


def gx_forward(y, kernel, alpha, rho_iters, denoise=None, trace=None):
    """models/unrolled_admm_gaussian.py:117-152 with the rhos given: [N,1,1,n] (SubNet) or [n].
    Returns z_n (the last denoiser output); ``trace`` receives x, z, u, rho lists (analysis=True)."""
    denoise = denoise if denoise is not None else (lambda t: t)
    y, Y, Ht, HtH = gx_spectra(y, kernel)
    z = gx_init_l2(Y, Ht, HtH, alpha)
    u = torch.zeros_like(y)
    n_iters = rho_iters.shape[-1]
    for i in range(n_iters):
        rho = rho_iters[:, :, :, i].view(-1, 1, 1, 1) if rho_iters.dim() == 4 else rho_iters[i]
        x = gx_x_update(Y, Ht, HtH, z, u, rho)
        z = denoise(rho * x + u)
        u = u + rho * (x - z)
        if trace is not None:
            for k, t in (("x", x), ("z", z), ("u", u), ("rho", rho)):
                trace.setdefault(k, []).append(t)
    return z


def normwise_error(out, ref):
    """Per-galaxy max|out - ref| / max|ref| (the parity metric of SURVEY.md 8(d)); returns [N]."""
    out = out.detach().double().cpu().reshape(out.shape[0], -1)
    ref = ref.detach().double().cpu().reshape(ref.shape[0], -1)
    return (out - ref).abs().amax(1) / ref.abs().amax(1).clamp_min(1e-300)


def pixel_error_floored(out, ref, floor=1e-5):
    """Per-galaxy max over pixels of |out - ref| / max(|ref|, floor * max|ref|): the per-pixel relative
    error with a floor (north_star's "1e-5 rel fp32 per pixel").  Pixels where the
    reference is ~0 are judged against floor * the galaxy's peak instead of their own magnitude.
    Returns [N]."""
    out = out.detach().double().cpu().reshape(out.shape[0], -1)
    ref = ref.detach().double().cpu().reshape(ref.shape[0], -1)
    den = torch.maximum(ref.abs(), floor * ref.abs().amax(1, keepdim=True)).clamp_min(1e-300)
    return ((out - ref).abs() / den).amax(1)


__all__ = ["psf_to_otf", "conv_fft_batch", "x_update", "v_update_poisson", "v_update_gaussian",
           "init_l2", "admm_forward", "wiener", "richardson_lucy", "tikhonov", "laplacian_kernel",
           "pad_double", "crop_half", "gx_spectra", "gx_init_l2", "gx_x_update", "gx_forward",
           "normwise_error", "pixel_error_floored"]

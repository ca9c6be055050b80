"""Reference-layout spectral helpers (``utils/utils_torch.py`` compatibility surface).

``psf_to_otf(ker, size)`` and ``conv_fft_batch(H, x)`` keep the reference's signatures and full
complex [N,1,H,W] OTF layout so existing callers work unchanged; internally they run on the HIP
engine's half-spectrum layout ([N, W//2+1, H], kx-major).  The layout conversions below are torch
tensor plumbing on the device; the transforms themselves are the engine's kernels.
"""
import torch
import torch.nn.functional as F

from . import engine


def half_to_full(otf_half, H, W):
    """[N, W//2+1, H] half spectrum -> full Hermitian spectrum [N, 1, H, W]."""
    N = otf_half.shape[0]
    K = W // 2 + 1
    half = otf_half.transpose(1, 2)                                # [N, H, K]  (ky, kx)
    full = torch.empty(N, H, W, dtype=otf_half.dtype, device=otf_half.device)
    full[:, :, :K] = half
    if W - K > 0:
        # X[ky, kx] = conj(X[-ky, W-kx]) for kx in [K, W)
        neg_ky = (-torch.arange(H, device=otf_half.device)) % H
        src = half[:, neg_ky][:, :, 1:W - K + 1].flip(-1)
        full[:, :, K:] = torch.conj(src)
    return full.view(N, 1, H, W)


def full_to_half(Hfull):
    """Full complex [N,1,H,W] spectrum -> Hermitian part restricted to kx <= W/2, as [N, K, H].

    conv_fft_batch takes the real part of the inverse FFT, which only sees the Hermitian part
    (H(k) + conj(H(-k)))/2 of H; for the OTF of a real PSF this is H itself."""
    Hf = Hfull.reshape(Hfull.shape[0], Hfull.shape[-2], Hfull.shape[-1]).to(torch.complex64)
    N, H, W = Hf.shape
    K = W // 2 + 1
    ky = (-torch.arange(H, device=Hf.device)) % H
    kx = (-torch.arange(K, device=Hf.device)) % W
    mirror = torch.conj(Hf[:, ky][:, :, kx])
    herm = 0.5 * (Hf[:, :, :K] + mirror)
    return herm.transpose(1, 2).contiguous()


def psf_to_otf(ker, size):
    """utils/utils_torch.py:79-92: returns (shifted zero-padded PSF [N,1,H,W], OTF [N,1,H,W] c64)."""
    N, _, H, W = size
    h = ker.shape[2]
    c = (h + 1) // 2
    psf = torch.zeros(size, dtype=torch.float32, device=ker.device)
    # same quadrant copy as the reference (PSF pixel (h/2, h/2) -> (0, 0))
    psf[:, :, :c, :c] = ker[:, :, c:, c:]
    psf[:, :, :c, -c:] = ker[:, :, c:, :c]
    psf[:, :, -c:, :c] = ker[:, :, :c, c:]
    psf[:, :, -c:, -c:] = ker[:, :, :c, :c]
    otf_half = engine.psf_to_otf_half(ker, N, H, W)
    return psf, half_to_full(otf_half, H, W)


def conv_fft_batch(H, x):
    """utils/utils_torch.py:46-50: Re IFFT2(FFT2(x) * H), H full-layout complex [N,1,H,W]."""
    return engine.conv_half(full_to_half(H), x)


def pad_double(img):
    """utils/utils_torch.py:11-13."""
    Hh, Ww = img.shape[-2], img.shape[-1]
    return F.pad(img, (Ww // 2, Ww // 2, Hh // 2, Hh // 2))


def crop_half(img):
    """utils/utils_torch.py:16-18."""
    Hh, Ww = img.shape[-2], img.shape[-1]
    return img[:, :, Hh // 4:3 * Hh // 4, Ww // 4:3 * Ww // 4]


__all__ = ["psf_to_otf", "conv_fft_batch", "half_to_full", "full_to_half", "pad_double", "crop_half"]

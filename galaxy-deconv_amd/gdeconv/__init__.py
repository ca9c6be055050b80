"""gdeconv - MI355X-native spectral engine for unrolled PnP-ADMM galaxy deconvolution.

Drop-in for the spectral hot path of mbertagna/Galaxy-Deconv: ``Unrolled_ADMM``, ``Wiener`` and
``Richard_Lucy`` keep the reference's ``nn.Module`` API (see ``gdeconv.models``); the FFT /
spectral-divide / dual-update work runs as hand-written HIP kernels for gfx950 behind the C ABI in
``include/gdeconv.h`` (``gdeconv/libgdeconv.so``).  Host plumbing, the ResUNet denoiser and the
SubNet stay in PyTorch-ROCm.
"""
from .nets import ResUNet, SubNet, ZUpdateResUNet  # noqa: F401
from .weights import make_state_dict  # noqa: F401


def __getattr__(name):  # engine-backed symbols load the HIP library lazily
    if name in ("Unrolled_ADMM", "Wiener", "Richard_Lucy"):
        from . import models
        return getattr(models, name)
    if name in ("psf_to_otf", "conv_fft_batch"):
        from . import spectral
        return getattr(spectral, name)
    raise AttributeError(name)

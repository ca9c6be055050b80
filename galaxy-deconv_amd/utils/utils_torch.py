"""Drop-in for reference ``utils/utils_torch.py`` hot-path helpers (``psf_to_otf`` :79-92,
``conv_fft_batch`` :46-50, ``pad_double`` :11-13, ``crop_half`` :16-18) on the HIP engine."""
from gdeconv.spectral import conv_fft_batch, crop_half, pad_double, psf_to_otf  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

"""Drop-in for reference ``models/XDenseUNet.py`` (PyTorch host-side denoiser)."""
from gdeconv.nets import XDenseUNet  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

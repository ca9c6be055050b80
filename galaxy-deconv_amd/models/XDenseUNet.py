"""Drop-in for reference ``models/XDenseUNet.py`` (PyTorch host-side denoiser)."""
from gdeconv.nets import XDenseUNet  # noqa: F401

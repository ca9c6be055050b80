"""Drop-in for reference ``models/unrolled_admm_gaussian.py`` (spectral steps + backward on the HIP engine)."""
from gdeconv.models import UnrolledADMMGaussian, XUpdateGaussian  # noqa: F401
from gdeconv.nets import SubNet, ZUpdateResUNet  # noqa: F401

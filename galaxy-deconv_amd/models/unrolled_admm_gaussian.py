"""Drop-in for reference ``models/unrolled_admm_gaussian.py`` (spectral steps + backward on the HIP engine)."""
from gdeconv.models import UnrolledADMMGaussian, XUpdateGaussian  # noqa: F401
from gdeconv.nets import SubNet, ZUpdateResUNet  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

"""Drop-in for reference ``models/Tikhonet.py`` (Tikhonov solve on the HIP engine)."""
from gdeconv.models import Tikhonet, Tikhonov  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

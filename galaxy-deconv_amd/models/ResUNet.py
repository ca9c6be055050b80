"""Drop-in for reference ``models/ResUNet.py`` (PyTorch; same module tree / state_dict keys)."""
from gdeconv.nets import ResUNet  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

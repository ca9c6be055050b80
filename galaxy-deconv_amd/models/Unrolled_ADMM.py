"""Drop-in for reference ``models/Unrolled_ADMM.py`` (``Unrolled_ADMM`` :153-215, ``SubNet`` :59-90)."""
from gdeconv.models import Unrolled_ADMM  # noqa: F401
from gdeconv.nets import SubNet, ZUpdateResUNet as Z_Update_ResUNet  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

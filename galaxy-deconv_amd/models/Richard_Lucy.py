"""Drop-in for reference ``models/Richard_Lucy.py``."""
from gdeconv.models import Richard_Lucy  # noqa: F401


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)

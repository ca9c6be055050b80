"""Drop-in for reference ``models/Wiener.py``."""
from gdeconv.models import Wiener  # noqa: F401

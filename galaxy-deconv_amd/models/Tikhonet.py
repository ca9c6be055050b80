"""Drop-in for reference ``models/Tikhonet.py`` (Tikhonov solve on the HIP engine)."""
from gdeconv.models import Tikhonet, Tikhonov  # noqa: F401

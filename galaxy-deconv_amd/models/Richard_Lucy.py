"""Drop-in for reference ``models/Richard_Lucy.py``."""
from gdeconv.models import Richard_Lucy  # noqa: F401

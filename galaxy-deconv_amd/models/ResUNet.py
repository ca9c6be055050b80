"""Drop-in for reference ``models/ResUNet.py`` (PyTorch; same module tree / state_dict keys)."""
from gdeconv.nets import ResUNet  # noqa: F401

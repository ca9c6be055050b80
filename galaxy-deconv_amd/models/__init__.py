"""Reference-path shims: with ``galaxy-deconv_amd`` on ``sys.path``,
``from models.Unrolled_ADMM import Unrolled_ADMM`` resolves to the HIP-backed drop-in exactly as
``test.py:12`` imports the reference."""
# modules this shim package does not provide import from the reference's package of the same name
from gdeconv import refpath as _refpath  # noqa: E402

__path__ = _refpath.extend(__path__, __name__)

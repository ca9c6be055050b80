"""Reference-path shims (``utils.utils_torch``, ``utils.utils_data``)."""
# modules this shim package does not provide import from the reference's package of the same name
from gdeconv import refpath as _refpath  # noqa: E402

__path__ = _refpath.extend(__path__, __name__)

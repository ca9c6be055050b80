"""Reference-path shims (``utils.utils_torch``)."""

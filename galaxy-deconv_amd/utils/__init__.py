"""Reference-path shims (``utils.utils_torch``, ``utils.utils_data``)."""

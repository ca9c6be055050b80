"""Fall-through from the drop-in shim packages (``models``, ``utils``) to the reference's own modules.

With ``galaxy-deconv_amd`` ahead of the reference checkout on ``sys.path``,
``models`` and ``utils`` resolve to this repository's shim packages.  Those override only the modules
on the accelerated path, so:

* ``extend(__path__, __name__)`` (called by the shims' ``__init__``) appends every other ``sys.path``
  entry's ``models/`` / ``utils/`` directory to the package path: modules the shims do not provide
  (``utils.utils_test``, ``utils.utils_train``, ``models.ADMMNet``, ...) import from the reference;
* ``attr(__name__, name)`` (each shim module's ``__getattr__``) serves names a shim module does not
  define (``models.Unrolled_ADMM.X_Update``, ``utils.utils_torch.conv_fft``, ...) from the reference's
  file of the same name, loaded once under a private module name (``_gdref.<module>``).

Nothing here is on the engine's compute path; it only keeps the reference's scripts importable.
"""
import importlib.util
import os
import pkgutil
import sys

_loaded = {}


def extend(path, name):
    return pkgutil.extend_path(path, name)


def reference_file(modname):
    """The reference's source file for ``modname`` (e.g. 'models.Unrolled_ADMM'), or None: the first
    package-path directory other than the shim's own that has it."""
    pkg, _, leaf = modname.rpartition(".")
    top = sys.modules.get(pkg)
    if top is None or not hasattr(top, "__path__"):
        return None
    mine = os.path.dirname(os.path.abspath(top.__file__)) if getattr(top, "__file__", None) else None
    for d in list(top.__path__):
        if mine is not None and os.path.abspath(d) == mine:
            continue
        f = os.path.join(d, leaf + ".py")
        if os.path.isfile(f):
            return f
    return None


def reference_module(modname):
    if modname in _loaded:
        return _loaded[modname]
    f = reference_file(modname)
    if f is None:
        raise ImportError(f"no reference module {modname!r} on sys.path")
    spec = importlib.util.spec_from_file_location("_gdref." + modname, f)
    mod = importlib.util.module_from_spec(spec)
    _loaded[modname] = mod           # before exec: tolerate import cycles through the shims
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del _loaded[modname]
        raise
    return mod


def attr(modname, name):
    """Module ``__getattr__`` of a shim: ``name`` from the reference's module of the same name."""
    if name.startswith("__"):
        raise AttributeError(name)
    try:
        mod = reference_module(modname)
    except ImportError as e:
        raise AttributeError(f"module {modname!r} has no attribute {name!r} (and no reference module to "
                             f"fall through to: {e})") from None
    try:
        return getattr(mod, name)
    except AttributeError:
        raise AttributeError(f"module {modname!r} has no attribute {name!r}") from None

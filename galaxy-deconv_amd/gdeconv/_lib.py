"""ctypes binding of ``libgdeconv.so`` (the C ABI declared in ``include/gdeconv.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``).
There is no fallback: if the library is missing or fails to load, every engine call raises.
``torch`` is imported first so that the process's single HIP runtime is torch's
``libamdhip64.so.7`` (the library's NEEDED entry resolves to the already-loaded soname).
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before dlopen of the engine)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgdeconv.so")

GD_OK = 0
ABI_VERSION = 5
GD_LLH = {"Gaussian": 0, "Poisson": 1}

_P = ctypes.c_void_p
_I = ctypes.c_int
_LL = ctypes.c_longlong
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); must match include/gdeconv.h exactly (checked by tests/test_abi.py)
SIGNATURES = {
    "gd_abi_version": (_I, []),
    "gd_engine_rev": (ctypes.c_char_p, []),
    "gd_engine_src_hash": (ctypes.c_char_p, []),
    "gd_hip_runtime_version": (_I, []),
    "gd_last_error": (ctypes.c_char_p, []),
    "gd_supported_size": (_I, [_I, _I]),
    "gd_workspace_bytes": (_SZ, [_I, _I, _I]),
    "gd_otf_bytes": (_SZ, [_I, _I, _I]),
    "gd_psf_to_otf": (_I, [_P, _LL, _I, _I, _I, _I, _I, _P, _P, _P]),
    "gd_conv_fft_batch": (_I, [_P, _I, _P, _P, _I, _I, _I, _P, _P]),
    "gd_conv_fft_batch_strided": (_I, [_P, _LL, _I, _P, _P, _I, _I, _I, _P, _P]),
    "gd_rfft2": (_I, [_P, _P, _I, _I, _I, _P]),
    "gd_irfft2": (_I, [_P, _P, _I, _I, _I, _P]),
    "gd_admm_state_bytes": (_SZ, [_I, _I, _I, _I]),
    "gd_admm_state_layout": (_I, [_I, _I, _I, _I]),
    "gd_admm_init_reads_rho": (_I, [_I, _I, _I]),
    "gd_admm_init": (_I, [_P, _P, _LL, _I, _I, _P, _LL, _P, _LL, _I, _I, _I, _I, _P, _P, _P, _P]),
    "gd_admm_iter": (_I, [_P, _P, _P, _P, _LL, _P, _LL, _P, _LL, _P, _LL, _I, _I, _I, _I, _I, _I, _P, _P,
                          _P]),
    "gd_admm_iter_v": (_I, [_P]),
    "gd_wiener": (_I, [_P, _P, _LL, _I, _I, _P, _LL, _P, _I, _I, _I, _P, _P]),
    "gd_richardson_lucy": (_I, [_P, _P, _LL, _I, _I, _I, _P, _I, _I, _I, _P, _P, _P]),
    "gd_tikhonov": (_I, [_P, _P, _LL, _I, _I, _P, _LL, _P, _LL, _P, _LL, _P, _I, _I, _I, _P, _P]),
    "gd_filter_power": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "gd_filter_power_taps": (_I, [_P, _P, _I, _P, _I, _I, _P]),
    "gd_gx_state_bytes": (_SZ, [_I, _I, _I]),
    "gd_gx_spec_bytes": (_SZ, [_I, _I, _I]),
    "gd_gx_init": (_I, [_P, _P, _LL, _I, _I, _P, _LL, _I, _I, _I, _P, _P, _P, _P]),
    "gd_gx_xupdate": (_I, [_P, _P, _P, _P, _LL, _P, _LL, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "gd_gx_xupdate_backward": (_I, [_P, _P, _P, _LL, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "gd_set_chunk_bytes": (_SZ, [_SZ]),
    "gd_set_pipeline_streams": (_I, [_I]),
    "gd_set_capture_pipeline": (_I, [_I]),
    "gd_set_fused_iteration": (_I, [_I]),
    "gd_set_fused_rl": (_I, [_I]),
    "gd_set_subnet_fused_max": (_I, [_I]),
    "gd_set_fused_init": (_I, [_I]),
    "gd_set_fused_min_batch": (_I, [_I, _I]),
    "gd_subnet_param_count": (_I, []),
    "gd_subnet_features": (_I, [_P, _P, _P, _I, _P]),
    "gd_subnet_mlp_param_count": (_I, [_I]),
    "gd_subnet_rhos": (_I, [_P, _P, _P, _P, _LL, _P, _P, _I, _I, _P]),
    "gd_subnet_rhos_psf": (_I, [_P, _LL, _I, _P, _P, _P, _LL, _P, _P, _I, _I, _P]),
    "gd_admm_init_subnet_supported": (_I, [_I, _I, _I, _I, _I, _I, _I]),
    "gd_admm_init_subnet": (_I, [_P, _P, _LL, _I, _I, _P, _LL, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P]),
    "gd_profile_enable": (_I, [_I]),
    "gd_profile_collect": (_I, []),
    "gd_profile_get": (_I, [_I, ctypes.c_char_p, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_LL)]),
    "gd_profile_reset": (_I, []),
    "gd_pack_open": (_I, [ctypes.c_char_p, ctypes.POINTER(_P), ctypes.POINTER(_LL), ctypes.POINTER(_I)]),
    "gd_pack_section_bytes": (_LL, [_P, _I]),
    "gd_pack_read": (_I, [_P, _I, _LL, _LL, _P, _I]),
    "gd_pack_gather": (_I, [_P, _I, _P, _LL, _P, _I]),
    "gd_pack_close": (_I, [_P]),
}

_lib = None

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def source_files():
    """The files the engine library is compiled from (the build's dependency list)."""
    import glob
    csrc = os.path.join(ROOT, "galaxy-deconv_amd", "csrc")
    return [os.path.join(csrc, "gd_engine.hip"), *sorted(glob.glob(os.path.join(csrc, "*.hpp"))),
            os.path.join(ROOT, "include", "gdeconv.h")]


# hipcc flags of the in-tree build (__graft_entry__.build); part of the provenance hash below, so a library
# built with other flags (offload arch, -D switches) is rebuilt and refused by smoke()
BUILD_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result"]


def _toolchain_id():
    """The ROCm release the build uses (/opt/rocm/.info/version; the same image on the GPU box)."""
    try:
        with open("/opt/rocm/.info/version") as f:
            return f.read().strip()
    except OSError:
        return "unknown"


def source_hash():
    """sha256 (first 16 hex digits) over the names and contents of ``source_files()``, the build flags and the
    ROCm release: what build() compiles into the library (``gd_engine_src_hash``) and smoke() checks against the
    tree it runs in."""
    import hashlib
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(("flags:" + " ".join(BUILD_FLAGS) + "\0rocm:" + _toolchain_id()).encode())
    return h.hexdigest()[:16]


class EngineError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load (once) and return the engine library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise EngineError(f"HIP engine library not found at {path}: build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gd_abi_version() != ABI_VERSION:
        raise EngineError("libgdeconv.so ABI version mismatch")
    _lib = lib
    return lib


def profile_enable(level=2):
    """0 off, 1 whole operations only, 2 operations + every kernel launch."""
    load().gd_profile_enable(int(level))


def profile_reset():
    load().gd_profile_reset()


def profile_collect():
    """{kernel name: (total_ms, launches)} accumulated since the last reset (synchronises)."""
    lib = load()
    n = lib.gd_profile_collect()
    if n < 0:
        check(n, "gd_profile_collect")
    out = {}
    buf = ctypes.create_string_buffer(128)
    for i in range(n):
        ms, cnt = ctypes.c_double(), _LL()
        check(lib.gd_profile_get(i, buf, 128, ctypes.byref(ms), ctypes.byref(cnt)), "gd_profile_get")
        out[buf.value.decode()] = (ms.value, cnt.value)
    return out


def check(rc, what):
    if rc != GD_OK:
        msg = load().gd_last_error()
        raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


__all__ = ["load", "check", "EngineError", "SIGNATURES", "LIB_PATH", "GD_LLH", "source_hash", "source_files"]

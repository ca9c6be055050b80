"""The C-ABI library loads (no GPU needed) and exports exactly what include/gdeconv.h declares,
with the ctypes binding's arity matching the header."""
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gdeconv.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(gd_\w+)\s*\(([^;]*?)\)\s*;", txt, flags=re.M | re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


@pytest.fixture(scope="module")
def lib():
    from gdeconv import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import importlib.util
        spec = importlib.util.spec_from_file_location("ge", os.path.join(ROOT, "__graft_entry__.py"))
        ge = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(ge)
        ge.build()
    return _lib.load()


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("gd_psf_to_otf", "gd_conv_fft_batch", "gd_admm_init", "gd_admm_iter", "gd_wiener",
                 "gd_richardson_lucy", "gd_rfft2", "gd_irfft2", "gd_last_error", "gd_workspace_bytes"):
        assert name in fns


def test_library_exports_every_header_symbol(lib):
    from gdeconv._lib import SIGNATURES
    fns = header_functions()
    assert set(fns) == set(SIGNATURES), "ctypes binding and header disagree"
    for name, nargs in fns.items():
        assert hasattr(lib, name), f"{name} not exported"
        assert len(SIGNATURES[name][1]) == nargs, f"{name}: header has {nargs} args"


def test_hip_runtime_version_is_torchs(lib):
    """In a PyTorch process the engine runs on the HIP runtime PyTorch bundles (same soname), not /opt/rocm's: the
    version gdeconv's capture guard reads (gd_hip_runtime_version) is torch.version.hip's."""
    import torch
    v = lib.gd_hip_runtime_version()
    assert v > 0
    if torch.version.hip:
        major, minor, patch = (int(x) for x in torch.version.hip.split(".")[:3])
        assert v == major * 10_000_000 + minor * 100_000 + patch


def test_host_only_queries(lib):
    from gdeconv import _lib as _lib_mod
    assert lib.gd_abi_version() == _lib_mod.ABI_VERSION == 5
    assert lib.gd_supported_size(256, 256) == 1 and lib.gd_supported_size(48, 48) == 1
    # other sizes up to 4096 per side, square or not, run the runtime-planned kernels (2)
    assert lib.gd_supported_size(50, 50) == 2 and lib.gd_supported_size(256, 128) == 2
    assert lib.gd_supported_size(48, 1025) == 2 and lib.gd_supported_size(1638, 1200) == 2
    assert lib.gd_supported_size(1639, 48) == 2 and lib.gd_supported_size(4096, 4096) == 2
    assert lib.gd_supported_size(1, 48) == 0 and lib.gd_supported_size(48, 4097) == 0
    # workspace: N * 2 images * (W/2+1) * H complex64
    assert lib.gd_workspace_bytes(4096, 256, 256) == 4096 * 2 * 129 * 256 * 8
    assert lib.gd_otf_bytes(2, 48, 48) == 2 * 25 * 48 * 8
    # UnrolledADMMGaussian's state on the 2H x 2W grid ([N][W+1][2H] |H|^2 fp32 + conj(H) Y complex64):
    # even sides, square or not (pad_double per axis); odd sides are unsupported, as in the reference
    assert lib.gd_gx_state_bytes(2, 40, 56) == 2 * 57 * 80 * 12
    assert lib.gd_gx_state_bytes(2, 48, 48) == 2 * 49 * 96 * 12
    assert lib.gd_gx_state_bytes(2, 41, 56) == 0 and lib.gd_gx_state_bytes(2, 40, 513) == 0


def test_switch_setters_are_strict(lib):
    """ABI 5: the fused-path setters take 0 or 1 only, the capture pipelining mode -1, 0 or 2 only; anything else
    is an error and leaves the setting unchanged (ABI 4 mapped any non-zero value to 1)."""
    for name in ("gd_set_fused_iteration", "gd_set_fused_init", "gd_set_fused_rl"):
        f = getattr(lib, name)
        cur = f(1)
        assert cur in (0, 1)
        assert f(2) == -1 and f(3) == -1 and f(-5) == -1
        assert f(cur) == 1, name              # still 1 after the refused values
    # 256^2: the chained kernels below these batches (Gaussian, Poisson, Richardson-Lucy); another op is an error
    assert [lib.gd_set_fused_min_batch(op, -1) for op in (0, 1, 2)] == [96, 192, 96]
    assert lib.gd_set_fused_min_batch(3, -1) == -1
    # the Poisson state layout at 256^2 follows the batch: two-pass (2) from 192 galaxies, three-kernel (3) below
    assert lib.gd_admm_state_layout(4096, 256, 256, 1) == 2 and lib.gd_admm_state_layout(64, 256, 256, 1) == 3
    assert lib.gd_admm_state_layout(64, 256, 256, 0) == 1 and lib.gd_admm_state_layout(1, 48, 48, 1) == 4
    assert lib.gd_set_capture_pipeline(1) == -2
    prev = lib.gd_set_capture_pipeline(2)
    assert prev in (-1, 0, 2)
    assert lib.gd_set_capture_pipeline(0) == 2
    assert lib.gd_set_capture_pipeline(prev) == 0


def test_argument_errors_need_no_device(lib):
    # validation happens before any HIP call: odd PSF, unsupported size, bad llh
    assert lib.gd_psf_to_otf(None, 0, 5, 5, 1, 48, 48, None, None, None) == -1
    assert b"even" in lib.gd_last_error()
    assert lib.gd_conv_fft_batch(None, 0, None, None, 1, 4097, 50, None, None) == -2
    assert lib.gd_admm_init(None, None, 0, 48, 48, None, 0, None, 0, 7, 1, 48, 48,
                            None, None, None, None) == -1
    # state: Gaussian |H|^2 (fp32) + conj(H)F(y/a) + F(u1) + conj(H)F(v-u2); Poisson OTF + two images
    assert lib.gd_admm_state_bytes(3, 48, 48, 0) == 3 * 25 * 48 * (4 + 3 * 8)
    assert lib.gd_admm_state_bytes(3, 48, 48, 1) == 3 * 25 * 48 * 8 + 2 * 3 * 48 * 48 * 4
    # an odd number of |H|^2 values is padded to keep the complex arrays 8-byte aligned
    assert lib.gd_admm_state_bytes(1, 45, 45, 0) == (23 * 45 + 1) // 2 * 8 + 3 * 23 * 45 * 8
    # at 256^2 the Gaussian slots are 256 KiB apart (HBM interleave spread, gd_engine.hip kStateSlotGap);
    # the Poisson layout stays packed
    spec = 3 * 129 * 256
    assert lib.gd_admm_state_bytes(3, 256, 256, 0) == (spec + 1) // 2 * 8 + 3 * spec * 8 + 3 * 256 * 1024
    assert lib.gd_admm_state_bytes(3, 256, 256, 1) == max(spec * 8 + 2 * 3 * 256 * 256 * 4,
                                                          spec * 4 + 4 * spec * 8 + 3 * 256 * 256 * 4)

"""Host-side logic that needs no GPU: module trees / state_dict compatibility, deterministic
weights, synthetic inputs, layout plumbing, argument validation."""
import json
import os

import pytest
import torch

import sys

from conftest import GOLDEN, ROOT


def test_state_dict_keys_match_reference():
    from gdeconv.models import Unrolled_ADMM
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))
    sd = Unrolled_ADMM(n_iters=8, llh="Gaussian").state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == ref
    assert len(sd) == 98


def test_subnet_false_parameters():
    from gdeconv.models import Unrolled_ADMM
    m = Unrolled_ADMM(n_iters=4, llh="Poisson", subnet=False)
    sd = m.state_dict()
    assert "rho1_iters" in sd and sd["rho2_iters"].shape == (4,)
    assert not any(k.startswith("init.") for k in sd)


def test_unsupported_variants_raise():
    from gdeconv.models import Unrolled_ADMM
    with pytest.raises(NotImplementedError):
        Unrolled_ADMM(PnP=False)
    with pytest.raises(ValueError):
        Unrolled_ADMM(llh="Laplace")


def test_xdenseunet_denoiser_selected_like_the_reference():
    """models/Unrolled_ADMM.py:163: ResUNet for 'ResUNet', XDenseUNet for any other name."""
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.nets import XDenseUNet, ResUNet
    assert isinstance(Unrolled_ADMM(n_iters=1, denoiser="XDenseUNet").Z.net, XDenseUNet)
    assert isinstance(Unrolled_ADMM(n_iters=1, denoiser="ResUNet").Z.net, ResUNet)


def test_unrolled_admm_is_inference_only():
    """Under autograd with trainable parameters the drop-in raises instead of silently returning an
    output with no graph to self.Z / self.init (the engine writes through raw pointers)."""
    from gdeconv.models import Unrolled_ADMM
    m = Unrolled_ADMM(n_iters=1, llh="Gaussian")
    x = torch.zeros(1, 1, 48, 48)
    with pytest.raises(NotImplementedError, match="inference-only"):
        m(x, torch.zeros(1, 1, 48, 48), torch.ones(1))
    # eval mode with grad enabled (figures/grid_plot.ipynb) runs under no_grad: on CPU tensors it gets as
    # far as the engine's device check
    m.eval()
    with pytest.warns(UserWarning, match="no_grad"), pytest.raises(ValueError, match="ROCm"):
        Unrolled_ADMM._warned_grad = False
        m(x, torch.zeros(1, 1, 48, 48), torch.ones(1))


def test_weights_deterministic_and_loadable():
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    m = Unrolled_ADMM(n_iters=2, llh="Gaussian")
    a, b = make_state_dict(m, 7), make_state_dict(m, 7)
    assert all(torch.equal(a[k], b[k]) for k in a)
    c = make_state_dict(m, 8)
    assert not torch.equal(a["Z.net.m_head.weight"], c["Z.net.m_head.weight"])
    m.load_state_dict(a)


def test_cpu_tensors_rejected_no_fallback():
    from gdeconv.models import Unrolled_ADMM, Wiener
    m = Unrolled_ADMM(n_iters=1, llh="Gaussian").eval()
    y, k, a = torch.rand(1, 1, 48, 48), torch.rand(1, 1, 48, 48), torch.ones(1, 1, 1, 1)
    with torch.no_grad(), pytest.raises(ValueError, match="ROCm"):
        m(y, k, a)
    with pytest.raises(ValueError, match="ROCm"):
        Wiener()(y, k, a)


def test_synth_batch_recipe():
    from gdeconv.synth import make_batch
    obs, psf, alpha, gt = make_batch(4, 48, seed=1)
    assert obs.shape == (4, 1, 48, 48) and psf.shape == (4, 1, 48, 48) and alpha.shape == (4, 1, 1, 1)
    assert torch.allclose(psf.sum((2, 3)), torch.full((4, 1), 1 / 16), rtol=1e-5)
    assert torch.allclose(alpha.view(-1), obs.flatten(1).mean(1), rtol=1e-5)
    o2, p2, a2, g2 = make_batch(4, 48, seed=1)
    assert torch.equal(obs, o2) and torch.equal(psf, p2)
    obs256, _, _, _ = make_batch(2, 256, seed=1)
    assert obs256.shape == (2, 1, 256, 256)


def test_half_full_layout_roundtrip():
    """Plumbing between the reference's full OTF layout and the engine's half layout."""
    from gdeconv.spectral import full_to_half, half_to_full
    for L in (48, 64):
        x = torch.rand(3, 1, L, L, dtype=torch.float64)
        full = torch.fft.fftn(x, dim=[2, 3]).to(torch.complex64)
        half = torch.fft.rfft2(x)[:, 0].transpose(1, 2).to(torch.complex64)
        assert torch.allclose(full_to_half(full), half, atol=1e-4)
        assert torch.allclose(half_to_full(half, L, L), full, atol=1e-4)


def test_shard_range_covers_batch():
    from gdeconv.dist import shard_range
    for N in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            parts = [shard_range(N, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == N
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def test_subnet_bn_folding_matches_reference_order():
    from gdeconv.nets import SubNet
    from gdeconv.weights import make_state_dict
    from gdeconv.synth import make_batch
    net = SubNet(8)
    net.load_state_dict(make_state_dict(net, 3))
    net.eval()
    _, psf, alpha, _ = make_batch(6, 64, seed=2)
    with torch.no_grad():
        a1, a2 = net.set_fold_bn(False)(psf, alpha)
        b1, b2 = net.set_fold_bn(True)(psf, alpha)
        c1, _ = net(psf, alpha)          # cached folded weights reused
    assert torch.allclose(a1, b1, rtol=2e-5, atol=1e-7) and torch.allclose(a2, b2, rtol=2e-5, atol=1e-7)
    assert torch.equal(b1, c1)


def test_subnet_engine_pack_layout():
    """The conv pack the engine SubNet kernels read (include/gdeconv.h): per layer the folded weights
    tap-major [cin][3][3][cout], then the bias [cout] (csrc/gd_subnet.hpp wtap)."""
    from gdeconv.nets import SubNet, _fold_conv_bn
    from gdeconv.weights import make_state_dict
    net = SubNet(4)
    net.load_state_dict(make_state_dict(net, 3))
    net.eval()
    pack = net._packed_params()
    pairs, _, _ = net._pack_modules()
    off = 0
    for conv, bn in pairs:
        w, b = _fold_conv_bn(conv, bn)
        co, ci = w.shape[:2]
        gen = torch.Generator().manual_seed(co * 100 + ci)
        for _ in range(25):
            c, i, dy, dx = (int(torch.randint(0, n, (1,), generator=gen)) for n in (co, ci, 3, 3))
            k = ((i * 3 + dy) * 3 + dx) * co + c
            assert pack[off + k] == w[c, i, dy, dx]
        off += co * ci * 9
        assert torch.equal(pack[off:off + co], b)
        off += co
    assert off == pack.numel() == 9196


def test_denoiser_micro_batching_is_transparent():
    """ZUpdateResUNet splits large batches into micro-batches (activations of a 4096 x 256^2 batch do
    not fit in HBM); per-galaxy results equal the one-call results (CPU, fp32), with and without
    autograd."""
    from gdeconv.nets import ZUpdateResUNet
    from gdeconv.weights import make_state_dict
    torch.manual_seed(0)
    z = ZUpdateResUNet(nc=(8, 16, 32, 64))
    z.load_state_dict(make_state_dict(z, 7))
    z.eval()
    x = torch.rand(5, 1, 24, 24)
    with torch.no_grad():
        full = z(x)
        z.micro_batch = 2
        part = z(x)
    assert torch.allclose(part, full, rtol=0, atol=1e-6 * float(full.abs().max()))
    xg = x.clone().requires_grad_(True)
    z(xg).sum().backward()
    z.micro_batch = None
    xf = x.clone().requires_grad_(True)
    z(xf).sum().backward()
    assert torch.allclose(xg.grad, xf.grad, rtol=0, atol=1e-6 * float(xf.grad.abs().max()))


REFERENCE = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "models")), reason="reference checkout absent")
def test_shims_fall_through_to_the_reference():
    """With the drop-ins ahead of the reference on sys.path, the
    reference's scripts still import: modules the shims do not provide resolve to the reference's
    files (test.py:15 utils.utils_test, train.py:15 utils.utils_train), names a shim module does not
    define come from the reference module (models.Unrolled_ADMM.X_Update, utils.utils_torch.conv_fft),
    and the accelerated classes stay the drop-ins.  Runs in a subprocess, bytecode writing off (the
    reference tree is read-only)."""
    import subprocess
    import sys
    code = r'''
import importlib.util, sys
sys.dont_write_bytecode = True
spec = importlib.util.find_spec("utils.utils_test")
assert spec is not None and spec.origin.startswith("/root/reference/"), spec
spec = importlib.util.find_spec("models.ADMMNet")
assert spec is not None and spec.origin.startswith("/root/reference/"), spec
import utils.utils_train as ut                       # imports utils.fit_ellipse from the reference
assert ut.__file__.startswith("/root/reference/")
from models.Unrolled_ADMM import Unrolled_ADMM, X_Update, Z_Update_XDenseUNet
import gdeconv.models
assert Unrolled_ADMM is gdeconv.models.Unrolled_ADMM
assert X_Update.__module__ == "_gdref.models.Unrolled_ADMM", X_Update.__module__
from utils.utils_torch import conv_fft_batch, conv_fft
import gdeconv.spectral
assert conv_fft_batch is gdeconv.spectral.conv_fft_batch and callable(conv_fft)
try:
    from models.Wiener import NoSuchName
except ImportError:
    pass
else:
    raise AssertionError("missing names must still raise")
print("ok")
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(repo, "galaxy-deconv_amd"), REFERENCE]),
               PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd="/tmp", capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_bench_rejects_world_size_mismatch():
    """A process group whose size is not --gpus exits non-zero before any GPU work (no mislabelled line)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--gpus 2" in r.stderr and not r.stdout.strip()

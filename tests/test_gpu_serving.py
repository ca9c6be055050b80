"""GPU tests for the serving-side rows of SURVEY 8(f) rank 2 (end-to-end denoiser throughput):
hipGraph capture of the whole unrolled forward (gdeconv.graphs) and the NHWC (channels_last)
ResUNet.  Bars: a replayed graph runs the same kernels as the eager forward, so its output is
bit-identical; the NHWC denoiser is fp32 like the NCHW one, so the full model stays within the
1e-5 normwise parity bar of the golden vectors (tests/golden/admm48.npz)."""
import numpy as np
import pytest
import torch

import admm_oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu
TOL = 1e-5
WEIGHT_SEED = 1234


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def nerr(out, ref):
    return float(O.normwise_error(out, ref).max())


def _model(n, llh, dev, identity=False):
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    m = Unrolled_ADMM(n_iters=n, llh=llh)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    m = m.to(dev).eval()
    if identity:
        m.Z = torch.nn.Identity()
    return m


@pytest.mark.parametrize("L,N", [(48, 37), (256, 5)])
@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
def test_graphed_forward_engine_bit_identical(dev, L, N, llh):
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    m = _model(8, llh, dev, identity=True)
    obs, psf, alpha, _ = make_batch(N, L, seed=9, device=dev)
    with torch.no_grad():
        eager = m(obs, psf, alpha)
    g = GraphedForward(m, obs, psf, alpha, clone=True)
    assert torch.equal(g(obs, psf, alpha), eager)
    # new inputs through the same graph
    obs2, psf2, alpha2, _ = make_batch(N, L, seed=10, device=dev)
    with torch.no_grad():
        eager2 = m(obs2, psf2, alpha2)
    assert torch.equal(g(obs2, psf2, alpha2), eager2)


@pytest.mark.parametrize("mode", [2, 0])
@pytest.mark.parametrize("H,W", [(100, 100), (90, 72)])
def test_graphed_forward_chunked_pipeline(dev, H, W, mode):
    """A forward whose runtime-planned operations run in several Infinity-Cache chunks (chunk bytes
    forced down to two galaxies; the 4096 x 160^2 bench line did the same at 96 MiB before 160^2 was fused)
    captures and replays bit-identically, with the chunks pipelined over the capturing thread's streams under
    capture (gd_set_capture_pipeline 2, GraphedForward's opt-in: an event set per operation) or in sequence (0,
    the engine's default; a mode the caller set is kept by GraphedForward)."""
    from gdeconv import _lib
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    lib = _lib.load()
    tgal = 2 * (W // 2 + 1) * H * 8
    old = lib.gd_set_chunk_bytes(2 * tgal)
    old_mode = lib.gd_set_capture_pipeline(mode)
    try:
        m = _model(8, "Gaussian", dev, identity=True)
        obs, psf, alpha, _ = make_batch(7, H, W, seed=11, device=dev)
        with torch.no_grad():
            eager = m(obs, psf, alpha)
        g = GraphedForward(m, obs, psf, alpha, clone=True)
        assert torch.equal(g(obs, psf, alpha), eager)
    finally:
        lib.gd_set_chunk_bytes(old)
        lib.gd_set_capture_pipeline(old_mode)


def test_graphed_forward_big_lines(dev):
    """Lines longer than 1638 points (dynamic LDS above 64 KiB, allowed per kernel at the eager warm-up): a 1700 x 1800
    forward captured and replayed bit-identically to the eager one."""
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    m = _model(2, "Gaussian", dev, identity=True)
    obs, psf, alpha, _ = make_batch(1, 1700, 1800, seed=17, device=dev)
    with torch.no_grad():
        eager = m(obs, psf, alpha)
    g = GraphedForward(m, obs, psf, alpha, clone=True)
    assert torch.equal(g(obs, psf, alpha), eager)


def test_graphed_forward_side_stream_chunked_init(dev):
    """The round-4 capture crash's shape, scaled down: a batch large enough for the init to run on a side stream
    beside the SubNet (models.CONCURRENT_INIT_PIXELS), the chunked runtime-planned Gaussian init (fused init off)
    in 6 chunks, captured and replayed bit-identically.  The side-stream init runs its chunks in sequence under
    capture (engine.ADMMState.init_concurrent), the iterations pipeline theirs."""
    from gdeconv import _lib
    from gdeconv.graphs import GraphedForward
    from gdeconv.models import CONCURRENT_INIT_PIXELS
    from gdeconv.synth import make_batch
    lib = _lib.load()
    H = W = 160
    N = -(-CONCURRENT_INIT_PIXELS // (H * W)) + 2
    tgal = 2 * (W // 2 + 1) * H * 8
    old = lib.gd_set_chunk_bytes((N // 6 + 1) * tgal)
    old_fi = lib.gd_set_fused_init(0)
    try:
        m = _model(8, "Gaussian", dev, identity=True)
        obs, psf, alpha, _ = make_batch(N, H, W, seed=13, device=dev)
        with torch.no_grad():
            eager = m(obs, psf, alpha)
        g = GraphedForward(m, obs, psf, alpha, clone=True)
        assert torch.equal(g(obs, psf, alpha), eager)
    finally:
        lib.gd_set_chunk_bytes(old)
        lib.gd_set_fused_init(old_fi)


def test_graphed_forward_full_model(dev):
    """Whole model incl. SubNet and the ResUNet denoiser, captured at 48^2."""
    from gdeconv.graphs import GraphedForward
    g0 = golden("admm48.npz")
    obs, psf, alpha = T(g0["obs"]).to(dev), T(g0["psf"]).to(dev), T(g0["alpha"]).to(dev)
    m = _model(2, "Gaussian", dev)
    with torch.no_grad():
        eager = m(obs, psf, alpha)
    g = GraphedForward(m, obs, psf, alpha, clone=True)
    out = g(obs, psf, alpha)
    # the engine's kernels replay bit-identically (tests above); MIOpen may pick another fp32
    # convolution algorithm for the captured ResUNet, so the whole model agrees to fp32 rounding
    assert nerr(out.cpu(), eager.cpu()) < 5e-6
    assert nerr(out.cpu(), T(g0["Gaussian_n2_out"])) < TOL


def test_graphed_forward_rejects_shape_change(dev):
    from gdeconv.graphs import GraphedForward
    from gdeconv.synth import make_batch
    m = _model(2, "Gaussian", dev, identity=True)
    obs, psf, alpha, _ = make_batch(4, 48, seed=1, device=dev)
    g = GraphedForward(m, obs, psf, alpha)
    with pytest.raises(ValueError):
        g(obs[:2], psf[:2], alpha[:2])


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
def test_channels_last_denoiser_parity(dev, llh):
    """NHWC ResUNet (the GPU default) against the NCHW one and the reference golden output."""
    g0 = golden("admm48.npz")
    obs, psf, alpha = T(g0["obs"]).to(dev), T(g0["psf"]).to(dev), T(g0["alpha"]).to(dev)
    m = _model(2, llh, dev)
    with torch.no_grad():
        out_cl = m(obs, psf, alpha).cpu()
        m.Z.net.channels_last = False
        m.Z.net.to(memory_format=torch.contiguous_format)
        out_nchw = m(obs, psf, alpha).cpu()
    assert nerr(out_cl, out_nchw) < 2e-6
    assert nerr(out_cl, T(g0[f"{llh}_n2_out"])) < TOL


# ------------------------------------------------------------------ packed ingest -> device batches
@pytest.fixture(scope="module")
def packed_golden(tmp_path_factory):
    from gdeconv.ingest import write_pack
    g = golden("ingest.npz")
    n_train = g["train_obs"].shape[0]
    p = str(tmp_path_factory.mktemp("pk") / "g.gdpack")
    write_pack(p, g["obs_raw"], g["psf_raw"], gt=g["gt_raw"],
               info={"n_total": 8, "n_train": n_train, "n_test": 8 - n_train, "sequence": list(range(8))})
    return p, g


@pytest.mark.parametrize("order", ["contiguous", "shuffled"])
def test_device_batches_match_reference_items(dev, packed_golden, order):
    """DeviceBatches (native reader -> pinned slots -> copy stream) delivers exactly the reference
    loader's items (bit-exact), in the drop-in's batch shapes."""
    from gdeconv.ingest import DeviceBatches, PackedGalaxies
    path, g = packed_golden
    ref = {k: np.concatenate([g[f"train_{k}"], g[f"test_{k}"]]) for k in ("obs", "psf", "alpha", "gt")}
    idx = np.arange(8) if order == "contiguous" else np.array([5, 2, 7, 0, 1, 6, 3, 4])
    with PackedGalaxies(path, threads=3) as pk:
        got = {k: [] for k in ref}
        for (obs, psf, alpha), gt in DeviceBatches(pk, 3, dev, indices=idx, with_gt=True):
            assert obs.is_cuda and obs.shape[1:] == (1, 48, 48) and alpha.shape[1:] == (1, 1, 1)
            for k, t in zip(("obs", "psf", "alpha", "gt"), (obs, psf, alpha, gt)):
                got[k].append(t.cpu().numpy())
    for k in ref:
        assert np.array_equal(np.concatenate(got[k]), ref[k][idx])


def test_device_batches_feed_the_engine(dev, packed_golden):
    from gdeconv.ingest import DeviceBatches, PackedGalaxies
    path, g = packed_golden
    m = _model(8, "Gaussian", dev, identity=True)
    r1 = torch.linspace(0.5, 1.5, 8, device=dev)  # fixed [n] rhos: no batch-size-dependent MLP GEMM
    r2 = torch.linspace(1.2, 0.3, 8, device=dev)
    m.rhos = lambda k, a: (r1, r2)
    outs = []
    with PackedGalaxies(path) as pk, torch.no_grad():
        for obs, psf, alpha in DeviceBatches(pk, 4, dev):
            outs.append(m(obs, psf, alpha))
        direct = m(torch.from_numpy(g["obs_raw"][:, None]).to(dev), torch.from_numpy(g["psf_raw"][:, None]).to(dev),
                   torch.from_numpy(np.concatenate([g["train_alpha"], g["test_alpha"]])).to(dev))
    assert torch.equal(torch.cat(outs), direct)


@pytest.mark.parametrize("N", [1, 37, 256, 1100])
def test_subnet_fused_launch_bit_identical(dev, N):
    """gd_subnet_rhos_psf: the one-launch per-galaxy SubNet (features + MLP in one workgroup, batches up
    to gd_set_subnet_fused_max) gives the same bits as the feature kernel + batched MLP kernel."""
    from gdeconv import _lib
    from gdeconv.synth import make_batch
    from gdeconv.weights import make_state_dict
    from models.Unrolled_ADMM import Unrolled_ADMM
    lib = _lib.load()
    m = Unrolled_ADMM(n_iters=8, llh="Gaussian")
    m.load_state_dict(make_state_dict(m, 1234))
    m = m.to(dev).eval()
    _, psf, alpha, _ = make_batch(N, 48, seed=900 + N, device=dev)
    old = lib.gd_set_subnet_fused_max(-1)
    outs = []
    try:
        for thr in (1 << 30, 0):
            lib.gd_set_subnet_fused_max(thr)
            with torch.no_grad():
                r1, r2 = m.init(psf, alpha)
            outs.append(torch.cat([r1.flatten(), r2.flatten()]).cpu())
    finally:
        lib.gd_set_subnet_fused_max(old)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])

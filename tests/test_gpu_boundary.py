"""Boundary robustness on the GPU: per-call workspaces on the caller's stream,
concurrent streams, the broadcast OTF of conv_fft_batch, argument validation, and the XDenseUNet
denoiser option of Unrolled_ADMM against a golden fixture made by the reference."""
import pytest
import torch

import admm_oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu
TOL = 1e-5


def T(a):
    return torch.from_numpy(a)


def nerr(a, b):
    return float(O.normwise_error(a, b).max())


def _batch(dev, N=24, L=64, seed=5):
    from gdeconv.synth import make_batch
    obs, psf, alpha, _ = make_batch(N, L, seed=seed, device=dev)
    return obs, psf, alpha


def test_two_streams_bit_identical_to_serial(dev):
    """Wiener, RL(5) and conv on two side streams at once (each call takes its scratch from the caching
    allocator on its own stream) give exactly the serial results."""
    from gdeconv import engine
    obs, psf, alpha = _batch(dev)
    otf = engine.psf_to_otf_half(psf, obs.shape[0], 64, 64)
    serial = (engine.wiener(obs, psf, alpha), engine.richardson_lucy(obs, psf, 5), engine.conv_half(otf, obs))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    res = {}
    for rep in range(3):
        with torch.cuda.stream(s1):
            res[("w", rep)] = engine.wiener(obs, psf, alpha)
            res[("c", rep)] = engine.conv_half(otf, obs)
        with torch.cuda.stream(s2):
            res[("r", rep)] = engine.richardson_lucy(obs, psf, 5)
            res[("w2", rep)] = engine.wiener(obs, psf, alpha)
    torch.cuda.synchronize()
    for rep in range(3):
        assert torch.equal(res[("w", rep)], serial[0])
        assert torch.equal(res[("w2", rep)], serial[0])
        assert torch.equal(res[("r", rep)], serial[1])
        assert torch.equal(res[("c", rep)], serial[2])


def test_two_host_threads_pipelined_calls(dev):
    """Two host threads issuing chunked (Infinity-Cache pipelined) operations at once, each on its own
    stream: the per-device fork / join events and internal streams are taken under a lock per call, so
    every result equals the serial one bit for bit."""
    import threading
    from gdeconv import _lib, engine
    from gdeconv.synth import make_batch
    lib = _lib.load()
    old = lib.gd_set_chunk_bytes(8 << 20)     # 15 galaxies of 256^2 per chunk -> many chunks per call
    try:
        obs, psf, alpha, _ = make_batch(40, 256, seed=31, device=dev)
        serial_w = engine.wiener(obs, psf, alpha)
        serial_c = engine.conv_half(engine.psf_to_otf_half(psf, 40, 256, 256), obs)
        torch.cuda.synchronize()
        res, errs = {}, []

        def work(tag):
            try:
                s = torch.cuda.Stream(dev)
                with torch.cuda.stream(s):
                    for rep in range(4):
                        res[(tag, "w", rep)] = engine.wiener(obs, psf, alpha)
                        res[(tag, "c", rep)] = engine.conv_half(engine.psf_to_otf_half(psf, 40, 256, 256), obs)
                s.synchronize()
            except Exception as e:  # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=work, args=(t,)) for t in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not errs, errs
        for t in range(2):
            for rep in range(4):
                assert torch.equal(res[(t, "w", rep)], serial_w)
                assert torch.equal(res[(t, "c", rep)], serial_c)
    finally:
        lib.gd_set_chunk_bytes(old)


def test_capture_pipeline_beside_eager_thread(dev):
    """One host thread captures a chunk-pipelined forward (gd_set_capture_pipeline 2, GraphedForward's opt-in)
    while a second thread runs eager chunk-pipelined calls INSIDE the capture window: the capture forks onto
    streams of the capturing thread, never the internal streams the eager calls use, so the eager kernels are
    not captured into the graph (nor invalidate it) and both results equal the serial ones bit for bit.  (The
    capture runs in torch's "thread_local" error mode: in "global" mode any potentially unsafe call of the other
    thread, the caching allocator's included, invalidates it whatever the engine does.)"""
    import threading
    from gdeconv import _lib, engine
    from gdeconv.graphs import GraphedForward
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.synth import make_batch
    lib = _lib.load()
    H = W = 100                                   # runtime-planned: chunked init / iterations
    tgal = 2 * (W // 2 + 1) * H * 8
    old = lib.gd_set_chunk_bytes(2 * tgal)
    try:
        obs, psf, alpha, _ = make_batch(7, H, W, seed=11, device=dev)
        wo, wp, wa, _ = make_batch(9, H, W, seed=12, device=dev)
        m = Unrolled_ADMM(n_iters=3, llh="Gaussian").to(dev).eval()
        with torch.no_grad():
            serial_w = engine.wiener(wo, wp, wa).clone()
        torch.cuda.synchronize()
        go, enq, ended = threading.Event(), threading.Event(), threading.Event()
        res, errs = [], []
        ws = torch.cuda.Stream(dev)

        def worker():
            try:
                with torch.cuda.stream(ws):       # warm the worker stream's allocator blocks before the capture
                    held = [engine.wiener(wo, wp, wa) for _ in range(3)]   # (no hipMalloc inside the window)
                    del held
                ws.synchronize()
                go.wait(60)
                with torch.cuda.stream(ws):
                    for _ in range(3):
                        res.append(engine.wiener(wo, wp, wa))
                enq.set()
                ended.wait(60)                     # no synchronising call while the capture is open
                ws.synchronize()
            except Exception as e:  # surfaced below
                errs.append(e)
                enq.set()

        class Gate(torch.nn.Module):                # the denoiser: holds the capture open while the worker enqueues
            def __init__(self):
                super().__init__()
                self.armed = False

            def forward(self, z):
                if self.armed and torch.cuda.is_current_stream_capturing():
                    self.armed = False
                    go.set()
                    enq.wait(60)
                return z

        m.Z = Gate()
        with torch.no_grad():
            eager = m(obs, psf, alpha).clone()   # (the gate is the identity outside a capture)
        t = threading.Thread(target=worker)
        t.start()
        m.Z.armed = True
        try:
            g = GraphedForward(m, obs, psf, alpha, clone=True, capture_error_mode="thread_local")
        finally:
            go.set()
            ended.set()
            t.join(120)
        assert not errs, errs
        assert len(res) == 3
        for r in res:
            assert torch.equal(r, serial_w)
        assert torch.equal(g(obs, psf, alpha), eager)
    finally:
        lib.gd_set_chunk_bytes(old)


def test_conv_fft_batch_shared_otf_broadcasts(dev):
    """conv_fft_batch(H, x) with ONE [1,1,H,W] OTF for N images (the reference's fftn(x) * H broadcast,
    utils/utils_torch.py:46-50): equal to the expanded per-galaxy OTF bit for bit, and to the oracle."""
    from gdeconv import engine
    from utils.utils_torch import conv_fft_batch, psf_to_otf
    obs, psf, _ = _batch(dev, N=7, L=48)
    _, H1 = psf_to_otf(psf[:1], (1, 1, 48, 48))
    out = conv_fft_batch(H1, obs)
    _, Hn = psf_to_otf(psf[:1].expand(7, 1, -1, -1).contiguous(), (7, 1, 48, 48))
    assert torch.equal(out, conv_fft_batch(Hn, obs))
    _, Ho = O.psf_to_otf(psf[:1].cpu(), (1, 1, 48, 48))
    ref = O.conv_fft_batch(Ho, obs.cpu())
    assert nerr(out.cpu(), ref) < TOL
    # the half-spectrum entry point broadcasts the same way
    otf1 = engine.psf_to_otf_half(psf[:1], 1, 48, 48)
    assert torch.equal(engine.conv_half(otf1, obs), out)


def test_conv_half_validates_the_otf(dev):
    from gdeconv import engine
    obs, psf, _ = _batch(dev, N=3, L=48)
    otf = engine.psf_to_otf_half(psf, 3, 48, 48)
    with pytest.raises(ValueError, match="complex64"):
        engine.conv_half(otf.to(torch.complex128), obs)
    with pytest.raises(ValueError):
        engine.conv_half(otf[:2], obs)                 # batch neither 1 nor N
    with pytest.raises(ValueError):
        engine.conv_half(otf[:, :10], obs)             # wrong spectrum shape
    with pytest.raises(ValueError):
        engine.conv_half(engine.psf_to_otf_half(psf, 3, 64, 64), obs)


def test_scalars_follow_the_input_device(dev):
    """Python-number alpha / lam are placed on the inputs' device (not the current one)."""
    from gdeconv import engine
    obs, psf, alpha = _batch(dev, N=2, L=48)
    a = float(alpha[0].item())
    x1 = engine.wiener(obs[:1], psf[:1], a)
    x2 = engine.wiener(obs[:1], psf[:1], alpha[:1])
    assert torch.equal(x1, x2)


def test_side_stream_state_path_matches_default_stream(dev):
    """A whole Unrolled_ADMM forward (init + iterations: per-call scratch, state buffer) enqueued on a
    side stream equals the default-stream forward."""
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    obs, psf, alpha = _batch(dev, N=5, L=48)
    m = Unrolled_ADMM(n_iters=3, llh="Gaussian")
    m.load_state_dict(make_state_dict(m, 3))
    m = m.to(dev).eval()
    m.Z = torch.nn.Identity()
    with torch.no_grad():
        a = m(obs, psf, alpha)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            b = m(obs, psf, alpha)
        torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("llh", ["Gaussian", "Poisson"])
def test_xdenseunet_denoiser_model_matches_reference(dev, llh):
    """Unrolled_ADMM(n_iters=2, denoiser='XDenseUNet') (models/Unrolled_ADMM.py:142-151, :163) on the
    GPU (HIP spectral path + PyTorch XDenseUNet / SubNet) against the reference's output
    (tests/golden/make_golden_r02.py)."""
    from gdeconv.models import Unrolled_ADMM
    from gdeconv.weights import make_state_dict
    g = golden("admm_xdense48.npz")
    m = Unrolled_ADMM(n_iters=2, llh=llh, denoiser="XDenseUNet")
    m.load_state_dict(make_state_dict(m, 1234))
    m = m.to(dev).eval()
    torch.backends.cudnn.allow_tf32 = False
    with torch.no_grad():
        out = m(T(g["obs"]).to(dev), T(g["psf"]).to(dev), T(g["alpha"]).to(dev)).cpu()
    e = nerr(out, T(g[f"{llh}_out"]))
    pix = float(O.pixel_error_floored(out, T(g[f"{llh}_out"])).max())
    print(f"xdense {llh}: normwise {e:.2e}, per-pixel (floor 1e-5 max|ref|) {pix:.2e}")
    assert e < TOL

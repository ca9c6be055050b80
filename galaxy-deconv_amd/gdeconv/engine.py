"""Tensor-level entry points of the HIP spectral engine (torch tensors in, torch tensors out).

Every function requires ROCm device tensors and enqueues the HIP kernels on torch's current
stream through the C ABI (``include/gdeconv.h``); nothing here computes on the CPU, and a missing
library raises (``gdeconv._lib.EngineError``).

Layouts: images fp32 [N,1,H,W] contiguous (NCHW, C=1, as in the reference); the OTF is the
half spectrum stored transposed, complex64 [N, W//2+1, H] (``otf[g, kx, ky]``).

Sizes: any H x W with 2 <= H, W <= 4096 (square or not).  Square 32/48/64/96/128/256 run the
compile-time-planned kernels (and the fused whole-galaxy kernels at 256^2 / <= 128); every other
size runs the runtime-planned kernels of ``csrc/gd_generic.hpp`` with the same operation chains
(``supported(H, W)`` returns 1 resp. 2).

Devices and streams: every entry point runs on the device of its (first) input tensor, under
``torch.cuda.device(that device)``, and enqueues on that device's current torch stream, whatever
the caller's current device is.  Scratch workspaces come from torch's caching allocator per call
(on that stream), so calls on different streams or threads never share scratch memory.
"""
import contextlib
import ctypes

import torch

from . import _lib


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)   # hipStream_t of (device index)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream(device=None):
    if _raw_stream is not None and device is not None and device.index is not None:
        return _raw_stream(device.index)
    return torch.cuda.current_stream(device).cuda_stream


def _current_device():
    return _cur_device() if _cur_device is not None else torch.cuda.current_device()


def _require_device(*ts):
    dev = None
    for t in ts:
        if t is None or not torch.is_tensor(t):
            continue
        if not t.is_cuda:
            raise ValueError("gdeconv runs on ROCm devices only: move tensors to 'cuda' "
                             "(the reference CPU path is not part of this engine)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"all tensors must be on one device (got {dev} and {t.device})")
    return dev


@contextlib.contextmanager
def _on(device):
    """Make ``device`` current for the duration of one engine call (the C side picks its internal
    pipeline streams by the current HIP device); no device switch when it already is."""
    if device.index is None or _current_device() == device.index:
        yield
        return
    with torch.cuda.device(device):
        yield


def _img(t, name):
    if t.dim() != 4 or t.shape[1] != 1:
        raise ValueError(f"{name} must be [N,1,H,W], got {tuple(t.shape)}")
    return t.float().contiguous()


def _galaxy_scalar(t, N, name, device=None):
    """(tensor, stride) for a per-galaxy scalar given as [N,1,1,1], [N], a 1-element tensor or a
    Python number (placed on ``device``, the call's device)."""
    if not torch.is_tensor(t):
        t = torch.tensor([float(t)], dtype=torch.float32, device=device if device is not None else "cuda")
    elif device is not None and t.device != torch.device(device):
        raise ValueError(f"{name} is on {t.device}, the inputs on {device}")
    t = t.float().contiguous().reshape(-1)
    if t.numel() == N:
        return t, 1
    if t.numel() == 1:
        return t, 0
    raise ValueError(f"{name} must have 1 or N={N} elements, got {t.numel()}")


def _psf(k, N, H, name="psf"):
    if k.dim() != 4 or k.shape[1] != 1:
        raise ValueError(f"{name} must be [N,1,h,w], got {tuple(k.shape)}")
    k = k.float().contiguous()
    if k.shape[0] not in (1, N):
        raise ValueError(f"{name} batch must be 1 or N={N}")
    gstride = 0 if k.shape[0] == 1 and N != 1 else k.shape[2] * k.shape[3]
    return k, gstride


_WS_BYTES = {}  # (N, H, W) -> gd_workspace_bytes (pure in its arguments; one ctypes call per shape)


def workspace(N, H, W, device):
    """Scratch of gd_workspace_bytes(N, H, W) bytes for ONE call, from torch's caching allocator on
    the current stream of ``device`` (freed back to that stream's pool when the caller drops it, so
    reuse is stream-ordered; nothing is shared across streams or threads)."""
    nbytes = _WS_BYTES.get((N, H, W))
    if nbytes is None:
        lib = _lib.load()
        if not lib.gd_supported_size(H, W):
            raise ValueError(f"unsupported image size {H}x{W} (H and W must be in [2, 4096])")
        nbytes = _WS_BYTES[(N, H, W)] = max(16, int(lib.gd_workspace_bytes(max(N, 1), H, W)))
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def empty_otf(N, H, W, device):
    return torch.empty(N, W // 2 + 1, H, dtype=torch.complex64, device=device)


def supported(H, W):
    """0 = unsupported, 1 = compile-time-planned size, 2 = runtime-planned (generic) size."""
    return int(_lib.load().gd_supported_size(H, W))


def psf_to_otf_half(psf, N, H, W):
    """Half-spectrum OTF [N, W//2+1, H] of ``psf_to_otf`` (utils/utils_torch.py:79-92)."""
    dev = _require_device(psf)
    lib = _lib.load()
    with _on(dev):
        k, gs = _psf(psf, N, H)
        otf = empty_otf(N, H, W, dev)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_psf_to_otf(k.data_ptr(), gs, k.shape[2], k.shape[3], N, H, W, otf.data_ptr(),
                                     ws.data_ptr(), _stream(dev)), "gd_psf_to_otf")
    return otf


def conv_half(otf_half, x, conj=False):
    """``conv_fft_batch(H, x)`` (utils/utils_torch.py:46-50) with H given as a half-spectrum OTF
    complex64 [1|N, W//2+1, H]; a 1-galaxy H applies to every image, as the reference's
    ``fftn(x) * H`` broadcasts a [1,1,H,W] H."""
    dev = _require_device(x, otf_half)
    lib = _lib.load()
    x = _img(x, "x")
    N, _, H, W = x.shape
    K = W // 2 + 1
    if otf_half.dtype != torch.complex64:
        raise ValueError(f"otf_half must be complex64, got {otf_half.dtype}")
    if otf_half.dim() != 3 or tuple(otf_half.shape[1:]) != (K, H) or otf_half.shape[0] not in (1, N):
        raise ValueError(f"otf_half must be [1|N={N}, {K}, {H}] for {H}x{W} images, got {tuple(otf_half.shape)}")
    otf_half = otf_half.contiguous()
    gstride = K * H if (otf_half.shape[0] == N and N > 1) else 0
    with _on(dev):
        out = torch.empty_like(x)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_conv_fft_batch_strided(otf_half.data_ptr(), gstride, int(conj), x.data_ptr(),
                                                 out.data_ptr(), N, H, W, ws.data_ptr(), _stream(dev)),
                   "gd_conv_fft_batch_strided")
    return out


def rfft2_half(x):
    """Half spectrum of real images, complex64 [N, W//2+1, H] (transposed), unnormalised."""
    dev = _require_device(x)
    lib = _lib.load()
    x = _img(x, "x")
    N, _, H, W = x.shape
    K = W // 2 + 1
    with _on(dev):
        spec = torch.empty(N, 2, K, H, dtype=torch.complex64, device=dev)
        _lib.check(lib.gd_rfft2(x.data_ptr(), spec.data_ptr(), N, H, W, _stream(dev)), "gd_rfft2")
    return spec[:, 0].contiguous()


def irfft2_half(spec, H, W):
    """Inverse of ``rfft2_half`` (normalised by 1/(H W)), fp32 [N,1,H,W]."""
    dev = _require_device(spec)
    lib = _lib.load()
    N, K = spec.shape[0], W // 2 + 1
    if spec.dtype != torch.complex64 or tuple(spec.shape[1:]) != (K, H):
        raise ValueError(f"spec must be complex64 [N, {K}, {H}], got {spec.dtype} {tuple(spec.shape)}")
    with _on(dev):
        buf = torch.zeros(N, 2, K, H, dtype=torch.complex64, device=dev)
        buf[:, 0] = spec
        out = torch.empty(N, 1, H, W, dtype=torch.float32, device=dev)
        _lib.check(lib.gd_irfft2(buf.data_ptr(), out.data_ptr(), N, H, W, _stream(dev)), "gd_irfft2")
    return out


def wiener(y, psf, alpha):
    """models/Wiener.py:10-20 on the HIP engine."""
    dev = _require_device(y, psf, alpha)
    lib = _lib.load()
    y = _img(y, "y")
    N, _, H, W = y.shape
    with _on(dev):
        k, gs = _psf(psf, N, H)
        al, al_s = _galaxy_scalar(alpha, N, "alpha", dev)
        out = torch.empty_like(y)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_wiener(y.data_ptr(), k.data_ptr(), gs, k.shape[2], k.shape[3], al.data_ptr(), al_s,
                                 out.data_ptr(), N, H, W, ws.data_ptr(), _stream(dev)), "gd_wiener")
    return out


def richardson_lucy(y, psf, n_iters):
    """models/Richard_Lucy.py:10-24 on the HIP engine."""
    dev = _require_device(y, psf)
    lib = _lib.load()
    y = _img(y, "y")
    N, _, H, W = y.shape
    with _on(dev):
        k, gs = _psf(psf, N, H)
        out = torch.empty_like(y)
        otf = empty_otf(N, H, W, dev)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_richardson_lucy(y.data_ptr(), k.data_ptr(), gs, k.shape[2], k.shape[3], int(n_iters),
                                          out.data_ptr(), N, H, W, otf.data_ptr(), ws.data_ptr(), _stream(dev)),
                   "gd_richardson_lucy")
    return out


def filter_power(filt):
    """|FFT2(filt)|^2 over the half spectrum, fp32 [N, W//2+1, H] (transposed like the OTF): the
    Tikhonov regulariser LtL of models/Tikhonet.py:26-27 from the placed filter image."""
    dev = _require_device(filt)
    lib = _lib.load()
    f = _img(filt, "filt")
    N, _, H, W = f.shape
    with _on(dev):
        out = torch.empty(N, W // 2 + 1, H, dtype=torch.float32, device=dev)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_filter_power(f.data_ptr(), out.data_ptr(), N, H, W, ws.data_ptr(), _stream(dev)),
                   "gd_filter_power")
    return out


def filter_power_taps(filt_img, device):
    """|FFT2|^2 over the half spectrum [1, W//2+1, H] of ONE sparse filter image (e.g. the placed
    Laplacian) by direct DFT in double on the device (gd_filter_power_taps).  The tap list of the
    constant image is extracted on the host (parameter setup, like weights)."""
    lib = _lib.load()
    device = torch.device(device)
    img = filt_img.detach().reshape(filt_img.shape[-2], filt_img.shape[-1]).float().cpu()
    H, W = img.shape
    nz = torch.nonzero(img)
    with _on(device):
        rc = nz.to(torch.int32).contiguous().to(device)
        vals = img[nz[:, 0], nz[:, 1]].contiguous().to(device)
        out = torch.empty(1, W // 2 + 1, H, dtype=torch.float32, device=device)
        _lib.check(lib.gd_filter_power_taps(rc.data_ptr() if len(nz) else None,
                                            vals.data_ptr() if len(nz) else None, int(len(nz)), out.data_ptr(),
                                            H, W, _stream(device)), "gd_filter_power_taps")
    return out


def tikhonov(y, psf, alpha, lam, ltl=None):
    """models/Tikhonet.py:15-31 (Tikhonov.forward) on the HIP engine: Re IFFT2(conj(H) FFT2(y/alpha) /
    (|H|^2 + lam LtL)); ``ltl`` None = filter 'Identity', else a half-spectrum [1|N, W//2+1, H]."""
    dev = _require_device(y, psf, alpha, lam, ltl)
    lib = _lib.load()
    y = _img(y, "y")
    N, _, H, W = y.shape
    with _on(dev):
        k, gs = _psf(psf, N, H)
        al, al_s = _galaxy_scalar(alpha, N, "alpha", dev)
        lm, lm_s = _galaxy_scalar(lam.detach() if torch.is_tensor(lam) else lam, N, "lam", dev)
        lptr, lgs = None, 0
        if ltl is not None:
            K = W // 2 + 1
            ltl = ltl.float().contiguous()
            if ltl.shape[-2:] != (K, H) or ltl.numel() not in (K * H, N * K * H):
                raise ValueError(f"ltl must be [1|N, {K}, {H}], got {tuple(ltl.shape)}")
            lptr, lgs = ltl.data_ptr(), (0 if ltl.numel() == K * H else K * H)
        out = torch.empty_like(y)
        ws = workspace(N, H, W, dev)
        _lib.check(lib.gd_tikhonov(y.data_ptr(), k.data_ptr(), gs, k.shape[2], k.shape[3], al.data_ptr(), al_s,
                                   lm.data_ptr(), lm_s, lptr, lgs, out.data_ptr(), N, H, W, ws.data_ptr(),
                                   _stream(dev)), "gd_tikhonov")
    return out


_MLP_COUNT = {}


def _mlp_param_count(n_out):
    c = _MLP_COUNT.get(n_out)
    if c is None:
        c = _MLP_COUNT[n_out] = int(_lib.load().gd_subnet_mlp_param_count(int(n_out)))
    return c


def _subnet_param_count():
    c = _MLP_COUNT.get("conv")
    if c is None:
        c = _MLP_COUNT["conv"] = int(_lib.load().gd_subnet_param_count())
    return c


def mlp_supported(n_out):
    """True if the engine's SubNet MLP kernels take ``n_out`` outputs (1 .. 64); larger MLPs (more than
    32 ADMM iterations) run the feature kernel and the PyTorch MLP."""
    return _mlp_param_count(n_out) > 0


def subnet_rhos(otf128, params, mlp_params, alpha, n_out):
    """The whole SubNet forward (``k_subnet_features`` + the batched ``k_subnet_mlp``: MLP, Softplus,
    + 1e-6) -> [N, n_out]; ``mlp_params`` packed (transposed weights) as documented in include/gdeconv.h,
    ``alpha`` [N] or one value."""
    dev = _require_device(otf128, params, mlp_params, alpha)
    lib = _lib.load()
    N = otf128.shape[0]
    if tuple(otf128.shape[1:]) != (65, 128) or otf128.dtype != torch.complex64:
        raise ValueError("otf128 must be complex64 [N, 65, 128]")
    if params.numel() != _subnet_param_count() or params.dtype != torch.float32:
        raise ValueError("bad SubNet parameter pack")
    if mlp_params.numel() != _mlp_param_count(int(n_out)) or mlp_params.dtype != torch.float32:
        raise ValueError("bad SubNet MLP parameter pack")
    al = alpha.reshape(-1).float().contiguous()
    if al.numel() not in (1, N):
        raise ValueError("alpha must hold 1 or N values")
    otf128 = otf128.contiguous()
    with _on(dev):
        out = torch.empty(N, int(n_out), dtype=torch.float32, device=dev)
        feat = torch.empty(N, 1024, dtype=torch.float32, device=dev)  # scratch (the features)
        _lib.check(lib.gd_subnet_rhos(otf128.data_ptr(), params.contiguous().data_ptr(), mlp_params.contiguous().data_ptr(),
                                      al.data_ptr(), 1 if al.numel() == N else 0, feat.data_ptr(), out.data_ptr(),
                                      int(n_out), N, _stream(dev)), "gd_subnet_rhos")
    return out


def subnet_rhos_psf(psf, params, mlp_params, alpha, n_out):
    """The whole SubNet forward from the PSFs (``k_subnet_features_psf``: |FFT2(pad128(psf))|^2 in the
    kernel, then the conv stack; ``k_subnet_mlp``) -> [N, n_out]; PSF side even and <= 64."""
    dev = _require_device(psf, params, mlp_params, alpha)
    lib = _lib.load()
    N = psf.shape[0]
    k, gs = _psf(psf, N, 128)
    h = k.shape[2]
    if k.shape[3] != h or h % 2 or h > 64:
        raise ValueError("subnet_rhos_psf needs an even square PSF of side <= 64")
    if params.numel() != _subnet_param_count() or params.dtype != torch.float32:
        raise ValueError("bad SubNet parameter pack")
    if mlp_params.numel() != _mlp_param_count(int(n_out)) or mlp_params.dtype != torch.float32:
        raise ValueError("bad SubNet MLP parameter pack")
    al = alpha.reshape(-1).float().contiguous()
    if al.numel() not in (1, N):
        raise ValueError("alpha must hold 1 or N values")
    with _on(dev):
        out = torch.empty(N, int(n_out), dtype=torch.float32, device=dev)
        feat = torch.empty(N, 1024, dtype=torch.float32, device=dev)  # scratch (the features)
        _lib.check(lib.gd_subnet_rhos_psf(k.data_ptr(), gs, h, params.contiguous().data_ptr(),
                                          mlp_params.contiguous().data_ptr(), al.data_ptr(), 1 if al.numel() == N else 0,
                                          feat.data_ptr(), out.data_ptr(), int(n_out), N, _stream(dev)),
                   "gd_subnet_rhos_psf")
    return out


def subnet_features(otf128, params):
    """SubNet conv features [N, 1024] from the 128x128 half-spectrum OTF of the PSFs
    (``k_subnet_features``; ``params`` packed as documented in include/gdeconv.h)."""
    dev = _require_device(otf128, params)
    lib = _lib.load()
    N = otf128.shape[0]
    if tuple(otf128.shape[1:]) != (65, 128) or otf128.dtype != torch.complex64:
        raise ValueError("otf128 must be complex64 [N, 65, 128]")
    if params.numel() != _subnet_param_count() or params.dtype != torch.float32:
        raise ValueError("bad SubNet parameter pack")
    otf128 = otf128.contiguous()
    with _on(dev):
        feat = torch.empty(N, 1024, dtype=torch.float32, device=dev)
        _lib.check(lib.gd_subnet_features(otf128.data_ptr(), params.contiguous().data_ptr(), feat.data_ptr(), N,
                                          _stream(dev)), "gd_subnet_features")
    return feat


class GaussXState:
    """Device state of one ``UnrolledADMMGaussian`` forward (models/unrolled_admm_gaussian.py:117-152):
    |H|^2 and G = F(max(y,0)) conj(H) on the 2x zero-padded grid (gd_gx_init), a private workspace.
    Images and PSFs are H x W (the PSF is padded like the image, so it must have the image's size)."""

    def __init__(self, y, psf, alpha):
        self.dev = _require_device(y, psf, alpha)
        self.lib = _lib.load()
        self.y = _img(y, "y")
        self.N, _, self.H, self.W = self.y.shape
        self.psf, self.psf_gs = _psf(psf, self.N, self.H)
        if tuple(self.psf.shape[-2:]) != (self.H, self.W):
            raise ValueError("UnrolledADMMGaussian pads the PSF like the image: psf must be H x W "
                             "(pad_double(kernel) at models/unrolled_admm_gaussian.py:122)")
        N1 = max(self.N, 1)
        nbytes = int(self.lib.gd_gx_state_bytes(N1, self.H, self.W))
        if nbytes == 0:
            raise ValueError(f"UnrolledADMMGaussian: unsupported image size {self.H}x{self.W} "
                             "(even sides 2 .. 2048: the 2x padded grid must fit the engine; the reference itself "
                             "fails on odd sides, its crop_half(pad_double(.)) returning H - 1 rows)")
        with _on(self.dev):
            self.alpha, self.alpha_s = _galaxy_scalar(alpha, self.N, "alpha", self.dev)
            self.state = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
            self.spec_bytes = int(self.lib.gd_gx_spec_bytes(N1, self.H, self.W))
            self.z0 = self._init()   # the state is valid from construction on

    def _ws(self):
        """Per-call scratch on the 2x padded grid (stream-ordered caching allocator)."""
        return workspace(self.N, 2 * self.H, 2 * self.W, self.dev)

    def init(self):
        """z0 = init_l2(Y, Ht, HtH, alpha) (:111-115), computed with the state at construction."""
        return self.z0

    def _init(self):
        z0 = torch.empty_like(self.y)
        k = self.psf
        _lib.check(self.lib.gd_gx_init(self.y.data_ptr(), k.data_ptr(), self.psf_gs, k.shape[2], k.shape[3],
                                       self.alpha.data_ptr(), self.alpha_s, self.N, self.H, self.W,
                                       self.state.data_ptr(), z0.data_ptr(), self._ws().data_ptr(),
                                       _stream(self.dev)), "gd_gx_init")
        return z0

    def rho(self, rho):
        return _galaxy_scalar(rho.detach() if torch.is_tensor(rho) else rho, self.N, "rho", self.dev)

    def x_update(self, z, u, rho, x_prev=None, rho_prev=None, zin=False, save=False):
        """x = XUpdateGaussian(Y, Ht, HtH, z, u, rho) (:85-93).  ``u`` None = 0.  ``x_prev`` given:
        u <- u + rho_prev (x_prev - z) in place first (the dual update :145 of the previous
        iteration).  Returns (x, rho x + u if zin, saved X spectrum if save)."""
        _require_device(z, u, x_prev, self.y)
        z = _img(z, "z")
        r, rs = self.rho(rho)
        if x_prev is not None:
            if u is None or rho_prev is None:
                raise ValueError("the fused dual update needs u and rho_prev")
            if not u.is_contiguous() or u.dtype != torch.float32:
                raise ValueError("u is updated in place: it must be contiguous fp32")
            x_prev = _img(x_prev, "x_prev")
        elif u is not None:
            u = _img(u, "u")
        rp, rps = self.rho(rho_prev) if rho_prev is not None else (None, 0)
        x = torch.empty_like(self.y)
        zi = torch.empty_like(self.y) if zin else None
        xs = torch.empty(self.spec_bytes, dtype=torch.uint8, device=self.y.device) if save else None
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        with _on(self.dev):
            _lib.check(self.lib.gd_gx_xupdate(z.data_ptr(), ptr(u), ptr(x_prev), r.data_ptr(), rs, ptr(rp), rps,
                                              x.data_ptr(), ptr(zi), ptr(xs), self.N, self.H, self.W,
                                              self.state.data_ptr(), self._ws().data_ptr(), _stream(self.dev)),
                       "gd_gx_xupdate")
        return x, zi, xs

    def x_backward(self, grad_x, z, rho, xs):
        """(dL/dz, dL/du, dL/drho [N]) of the X update from dL/dx (self-adjoint linear part)."""
        g = _img(grad_x, "grad_x")
        z = _img(z, "z")
        r, rs = self.rho(rho)
        gz, gu = torch.empty_like(self.y), torch.empty_like(self.y)
        part = torch.empty(self.N, self.W + 1, dtype=torch.float32, device=self.y.device)
        with _on(self.dev):
            _lib.check(self.lib.gd_gx_xupdate_backward(g.data_ptr(), z.data_ptr(), r.data_ptr(), rs, xs.data_ptr(),
                                                       gz.data_ptr(), gu.data_ptr(), part.data_ptr(), self.N, self.H,
                                                       self.W, self.state.data_ptr(), self._ws().data_ptr(),
                                                       _stream(self.dev)), "gd_gx_xupdate_backward")
        return gz, gu, part.sum(1)


class _XUpdateGaussianFn(torch.autograd.Function):
    """Autograd of XUpdateGaussian on the engine: x = M (rho z - u) + b(rho) with M self-adjoint, so
    dz = rho M g, du = -M g, drho = <g, C IFFT((F(pad z) - X) / (rho + HtH))> (gd_gx_xupdate_backward)."""

    @staticmethod
    def forward(ctx, z, u, rho, st):
        x, _, xs = st.x_update(z.detach(), u.detach(), rho, save=True)
        ctx.st, ctx.xs = st, xs
        ctx.rho_shape = rho.shape if torch.is_tensor(rho) else None
        ctx.save_for_backward(z.detach().float().contiguous(), rho if torch.is_tensor(rho) else torch.tensor(rho))
        return x

    @staticmethod
    def backward(ctx, gx):
        z, rho = ctx.saved_tensors
        st = ctx.st
        gz, gu, grho = st.x_backward(gx.contiguous(), z, rho, ctx.xs)
        gr = None
        if ctx.needs_input_grad[2]:
            gr = (grho.sum() if rho.numel() == 1 else grho).reshape(ctx.rho_shape).to(rho.dtype)
        return (gz if ctx.needs_input_grad[0] else None, gu if ctx.needs_input_grad[1] else None, gr, None)


def gx_x_update(st, z, u, rho):
    """Differentiable X update of UnrolledADMMGaussian (autograd through the HIP backward)."""
    return _XUpdateGaussianFn.apply(z, u, rho, st)


class RhoSchedule:
    """Per-iteration (device pointer, galaxy stride) pairs of a penalty schedule, computed once per
    forward: a [N', 1, 1, n] SubNet output (N' = N, or 1 = shared; any view whose last dim is unit
    stride, e.g. the rho1 / rho2 halves of the MLP output) or an [n] parameter.  No per-iteration slicing
    or tensor creation: iteration ``it`` is ``base + 4 it`` (models/Unrolled_ADMM.py:201-206 index
    ``rho1_iters[:, :, :, n]``)."""

    __slots__ = ("t", "base", "gs", "n")

    def __init__(self, rho_iters, N, device):
        t = rho_iters.detach()
        if t.dtype != torch.float32:
            t = t.float()
        if t.device != torch.device(device):
            raise ValueError(f"rho schedule is on {t.device}, the inputs on {device}")
        if t.dim() == 4:
            t = t.reshape(t.shape[0], t.shape[-1]) if t.shape[1] == 1 and t.shape[2] == 1 else None
            if t is None:
                raise ValueError("rho schedule must be [N,1,1,n]")
            if t.stride(1) != 1:
                t = t.contiguous()
            if t.shape[0] not in (1, N):
                raise ValueError(f"rho schedule batch must be 1 or N={N}")
            self.gs = t.stride(0) if (t.shape[0] == N and N > 1) else 0
            self.n = t.shape[1]
        elif t.dim() == 1:
            t = t.contiguous()
            self.gs, self.n = 0, t.shape[0]
        else:
            raise ValueError("rho schedule must be [N,1,1,n] or [n]")
        self.t, self.base = t, t.data_ptr()

    def __getitem__(self, it):
        if not 0 <= it < self.n:
            raise IndexError(f"iteration {it} outside the schedule of {self.n}")
        return self.base + 4 * it, self.gs


def _scalar_arg(x, dev):
    """(pointer, stride) from a (tensor | device pointer, stride) pair."""
    p, s = x
    if torch.is_tensor(p):
        if p.device != dev:
            raise ValueError(f"per-galaxy scalar on {p.device}, the inputs on {dev}")
        if p.dtype != torch.float32:
            raise ValueError("per-galaxy scalars must be fp32")
        return p.data_ptr(), s
    return int(p), s


_NESTED_FORK_SAFE = None


def _nested_capture_fork_safe(lib):
    """True when the HIP runtime this process runs on captures a fork from a non-origin capture stream (ROCm >= 7.2;
    7.0, which PyTorch 2.10+rocm7.0 bundles, segfaults in hipStreamEndCapture on it)."""
    global _NESTED_FORK_SAFE
    if _NESTED_FORK_SAFE is None:
        _NESTED_FORK_SAFE = lib.gd_hip_runtime_version() >= 70200000
    return _NESTED_FORK_SAFE


class ADMMState:
    """Device state of one unrolled-ADMM forward: the engine's opaque state buffer (OTF + u1 and
    v - u2, spectral for llh='Gaussian', spatial for 'Poisson'), ``zin``, the next denoiser input
    (x + u1), and the call scratch.  Everything is allocated once at construction (on the current
    stream of the inputs' device) and reused by ``init`` and every ``step``, which are stream-ordered
    on that stream like the state itself; a step validates only what changes per call (z, the output),
    so the host cost per iteration is one ctypes call (the 48^2 LSST batch is host-launch-bound)."""

    def __init__(self, y, psf, alpha, llh):
        self.dev = _require_device(y, psf, alpha)
        self.lib = _lib.load()
        self.y = _img(y, "y")
        self.N, _, self.H, self.W = self.y.shape
        self.psf, self.psf_gs = _psf(psf, self.N, self.H)
        if llh not in _lib.GD_LLH:
            raise ValueError("llh must be 'Gaussian' or 'Poisson'")
        self.llh = _lib.GD_LLH[llh]
        skey = (self.N, self.H, self.W, self.llh)
        nbytes = ADMMState._state_bytes.get(skey)
        if nbytes is None:
            if not self.lib.gd_supported_size(self.H, self.W):
                raise ValueError(f"unsupported image size {self.H}x{self.W} (H and W must be in [2, 4096])")
            nbytes = ADMMState._state_bytes[skey] = int(self.lib.gd_admm_state_bytes(max(self.N, 1), self.H, self.W,
                                                                                      self.llh))
        with _on(self.dev):
            self.alpha, self.alpha_s = _galaxy_scalar(alpha, self.N, "alpha", self.dev)
            self.state = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
            self.zin = torch.empty_like(self.y)
            self.ws = workspace(self.N, self.H, self.W, self.dev)
        self._fixed = (self.y.data_ptr(), self.alpha.data_ptr(), self.alpha_s, self.state.data_ptr(),
                       self.ws.data_ptr())
        self._dev_index = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        self._shape = tuple(self.y.shape)
        self._bind()
        self.layout = None
        self.iter = 0
        self._side = None   # the _side_streams entry an init_concurrent() is running on, until joined
        # not cached: for Poisson it follows the fused-path switches (state layout 4: iteration 0 forms w1);
        # _reads_rho holds overrides only (tests force the serial order with it)
        r = ADMMState._reads_rho.get((self.H, self.W, self.llh))
        if r is None:
            r = int(self.lib.gd_admm_init_reads_rho(self.H, self.W, self.llh))
        self.init_reads_rho = r > 0

    _reads_rho = {}     # (H, W, llh) -> forced gd_admm_init_reads_rho (overrides for tests; empty by default)
    _state_bytes = {}   # (N, H, W, llh) -> gd_admm_state_bytes (pure in its arguments)
    # (device index, main stream) -> (side stream, fork event, join event) of init_concurrent (LRU, bounded).  The fork
    # and join go through these persistent events rather than Stream.wait_stream's temporary ones (one event pair per
    # side stream, no event created or destroyed per forward; whether the events are temporary made no difference to
    # the ROCm 7.0 capture crash, profiles/r06_capture_rootcause.txt)
    _side_streams = {}
    _SIDE_STREAMS_MAX = 16

    @property
    def otf(self):
        """Half-spectrum OTF [N, W//2+1, H] (Poisson state only; the Gaussian state keeps |H|^2 and
        conj(H) F(y/alpha) instead)."""
        if self.llh != _lib.GD_LLH["Poisson"]:
            raise AttributeError("the Gaussian ADMM state stores |H|^2, not the OTF")
        K = self.W // 2 + 1
        return self.state[: self.N * K * self.H * 8].view(torch.complex64).view(self.N, K, self.H)

    def init(self, rho2_first):
        """models/Unrolled_ADMM.py:181-196 + init_l2 + the first V step; ``rho2_first`` = (tensor or
        device pointer, stride), or None when the init reads no rho (``init_reads_rho`` False: Gaussian)."""
        if rho2_first is None:
            if self.init_reads_rho:
                raise ValueError("this init takes the first V step: it needs rho2_first")
            r2, r2s = None, 0
        else:
            r2, r2s = _scalar_arg(rho2_first, self.dev)
        k = self.psf
        yp, ap, as_, sp, wp = self._fixed
        with _on(self.dev):
            _lib.check(self.lib.gd_admm_init(
                yp, k.data_ptr(), self.psf_gs, k.shape[2], k.shape[3], ap, as_, r2, r2s, self.llh, self.N, self.H,
                self.W, sp, self.zin.data_ptr(), wp, _stream(self.dev)), "gd_admm_init")
        self.layout = self.lib.gd_admm_state_layout(self.N, self.H, self.W, self.llh)
        self.iter = 0

    def init_with_subnet(self, params, mlp_params, n_out):
        """``init`` and the engine SubNet (``subnet_rhos_psf`` of this state's PSFs and alphas; packs from
        ``SubNet.engine_packs``) in ONE launch (gd_admm_init_subnet: small stamps, small batches, Gaussian)
        -> the rhos [N, n_out], bit-identical to the two separate calls; None when the pair is not fusable
        here (the caller then runs the SubNet and ``init`` / ``init_concurrent``)."""
        if self.init_reads_rho:
            return None
        k = self.psf
        if not self.lib.gd_admm_init_subnet_supported(self.N, self.H, self.W, k.shape[2], k.shape[3], self.llh,
                                                      int(n_out)):
            return None
        if params.numel() != _subnet_param_count() or params.dtype != torch.float32 or params.device != self.dev:
            raise ValueError("bad SubNet parameter pack")
        if mlp_params.numel() != _mlp_param_count(int(n_out)) or mlp_params.dtype != torch.float32 \
                or mlp_params.device != self.dev:
            raise ValueError("bad SubNet MLP parameter pack")
        yp, ap, as_, sp, wp = self._fixed
        with _on(self.dev):
            rhos = torch.empty(self.N, int(n_out), dtype=torch.float32, device=self.dev)
            _lib.check(self.lib.gd_admm_init_subnet(
                yp, k.data_ptr(), self.psf_gs, k.shape[2], k.shape[3], ap, as_, self.llh, self.N, self.H, self.W, sp,
                self.zin.data_ptr(), params.contiguous().data_ptr(), mlp_params.contiguous().data_ptr(),
                rhos.data_ptr(), int(n_out), wp, _stream(self.dev)), "gd_admm_init_subnet")
        self.layout = self.lib.gd_admm_state_layout(self.N, self.H, self.W, self.llh)
        self.iter = 0
        return rhos

    def init_concurrent(self):
        """The init (Gaussian: it reads no rho) on a side stream forked from the device's current
        stream, so that it runs while the caller enqueues the SubNet on the current stream (at 48^2 both
        are one latency-bound round of workgroups that fit on a CU together).  The first ``step`` (or
        ``join``) makes the current stream wait for it; graph-capturable (event fork / join)."""
        if self.init_reads_rho:
            raise ValueError("this init takes the first V step: it needs the rhos (use init(rho2_first))")
        main = torch.cuda.current_stream(self.dev)
        # one side stream per (device, caller's stream): two host threads forwarding on their own streams
        # do not serialise their inits on a shared side stream (nor join each other's); a bounded cache, so
        # the streams of callers that come and go are not kept forever
        key = (self._dev_index, main.cuda_stream)
        entry = ADMMState._side_streams.pop(key, None)
        if entry is None:
            entry = (torch.cuda.Stream(device=self.dev), torch.cuda.Event(), torch.cuda.Event())
        ADMMState._side_streams[key] = entry         # most recently used last
        while len(ADMMState._side_streams) > ADMMState._SIDE_STREAMS_MAX:
            ADMMState._side_streams.pop(next(iter(ADMMState._side_streams)))
        side, fork, _ = entry
        fork.record(main)
        side.wait_event(fork)
        # under stream capture a chunked init on the side stream runs its chunks in sequence on HIP runtimes before
        # 7.2: there a fork from a stream that joined the capture through an event (the side stream) onto other
        # streams segfaults inside hipStreamEndCapture - a runtime bug, reproduced without the engine by
        # tools/capture_probe.hip mode 2 on PyTorch's bundled ROCm 7.0 runtime and absent on ROCm 7.2's
        # (profiles/r06_capture_rootcause.txt)
        serial = torch.cuda.is_current_stream_capturing() and not _nested_capture_fork_safe(self.lib)
        old = self.lib.gd_set_capture_pipeline(0) if serial else None
        try:
            with torch.cuda.stream(side):
                self.init(None)
        finally:
            if serial:
                self.lib.gd_set_capture_pipeline(old)
        self._side = entry

    def join(self):
        """Make the device's current stream wait for an ``init_concurrent`` (no-op otherwise)."""
        if self._side is not None:
            side, _, ev = self._side
            ev.record(side)
            torch.cuda.current_stream(self.dev).wait_event(ev)
            self._side = None

    def _bind(self):
        """The packed argument vector of gd_admm_iter_v (its 20 slots in gd_admm_iter's order): the slots fixed for
        this state (y, alpha, llh, N, H, W, state, workspace) set here from ``_fixed``, the per-call ones by ``step``
        (one 1-argument ctypes call per iteration instead of 20 converted arguments: the eager 256 x 48^2 forward is
        host-bound).  Call again after re-pointing ``_fixed``."""
        yp, ap, as_, sp, wp = self._fixed
        v = self._argv = (ctypes.c_longlong * 20)()
        v[0], v[3], v[4], v[11] = yp, ap, as_, self.llh
        v[14], v[15], v[16], v[17], v[18] = self.N, self.H, self.W, sp, wp
        self._argv_addr = ctypes.addressof(v)
        self._iter_v = self.lib.gd_admm_iter_v

    def step(self, z, rho1, rho2, rho2_next, out=None):
        """One loop body (models/Unrolled_ADMM.py:207-213) after the denoiser returned ``z``.
        ``rho*`` are (tensor or device pointer, stride) pairs (``RhoSchedule`` items); ``rho2_next`` None
        marks the last iteration, whose x (times alpha for Poisson) goes to ``out``."""
        if self.layout is None:
            raise _lib.EngineError("ADMMState.step before init")
        if self._side is not None:
            self.join()
        if z.dtype != torch.float32 or not z.is_contiguous():
            z = z.float().contiguous()
        if z.shape != self._shape:
            raise ValueError(f"denoiser returned {tuple(z.shape)}, expected {self._shape}")
        if z.device != self.dev:
            raise ValueError(f"denoiser returned a tensor on {z.device}, the state is on {self.dev}")
        last = rho2_next is None
        if last:
            if out is None or out.shape != self._shape or out.dtype != torch.float32 or out.device != self.dev \
                    or not out.is_contiguous():
                raise ValueError("the last iteration needs a contiguous fp32 `out` shaped like y on the state's device")
            dst = out
        else:
            dst = self.zin
        if self.llh != 0 and self.lib.gd_admm_state_layout(self.N, self.H, self.W, self.llh) != self.layout:
            raise _lib.EngineError("the ADMM state layout changed since init (gd_set_fused_iteration toggled "
                                   "between gd_admm_init and gd_admm_iter)")
        v = self._argv
        v[5], v[6] = _scalar_arg(rho1, self.dev)
        v[7], v[8] = _scalar_arg(rho2, self.dev)
        if last:
            v[9], v[10] = 0, 0
        else:
            v[9], v[10] = _scalar_arg(rho2_next, self.dev)
        v[1], v[2], v[12], v[13] = z.data_ptr(), dst.data_ptr(), self.iter, last
        if _current_device() == self._dev_index:
            v[19] = _stream(self.dev) or 0
            rc = self._iter_v(self._argv_addr)
        else:
            with _on(self.dev):
                v[19] = _stream(self.dev) or 0
                rc = self._iter_v(self._argv_addr)
        if rc:
            _lib.check(rc, "gd_admm_iter")
        self.iter += 1
        return dst


__all__ = ["psf_to_otf_half", "conv_half", "rfft2_half", "irfft2_half", "wiener", "richardson_lucy",
           "tikhonov", "filter_power", "filter_power_taps", "GaussXState", "gx_x_update",
           "ADMMState", "RhoSchedule", "workspace", "empty_otf", "supported", "subnet_features", "subnet_rhos", "subnet_rhos_psf",
           "mlp_supported"]

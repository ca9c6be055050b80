"""Drop-in ``nn.Module``s with the reference's API, running the spectral path on the HIP engine.

* ``Unrolled_ADMM(n_iters=8, llh='Poisson', denoiser='ResUNet', PnP=True, subnet=True)`` -
  same constructor, attributes and ``state_dict`` keys as ``models/Unrolled_ADMM.py:153-215``
  (98 keys with the SubNet; ``rho1_iters``/``rho2_iters`` parameters with ``subnet=False``), same
  ``forward(y, kernel, alpha)`` semantics.  The ResUNet denoiser (``self.Z``) and the SubNet
  (``self.init``) stay in PyTorch; every spectral step goes through ``gdeconv.engine``.
* ``Wiener().forward(y, psf, alpha)`` - ``models/Wiener.py:10-20``.
* ``Richard_Lucy(n_iters).forward(y, psf)`` - ``models/Richard_Lucy.py:10-24``.
* ``UnrolledADMMGaussian(n_iters=8, denoiser='ResUNet', PnP=True, subnet=True, analysis=False)`` -
  ``models/unrolled_admm_gaussian.py:96-152`` (the variant ``train.py:41`` trains): spectral steps
  on the engine with a HIP backward for training; ResUNet(nc=32..256) and its SubNet in PyTorch.
* ``Tikhonov(filter).forward(y, psf, alpha, lam)`` / ``Tikhonet(filter)`` - ``models/Tikhonet.py:8-47``
  (the Tikhonov solve on the engine, the XDenseUNet denoiser in PyTorch).

Differences from the reference, all deliberate: the device is taken from the input (the reference
hard-codes ``cuda:0``, ``models/Unrolled_ADMM.py:178``), the OTF is computed on the device (the
reference builds it on the CPU every forward, ``utils/utils_torch.py:81``), CPU tensors are
rejected (no CPU path), unsupported reference variants raise instead of misbehaving
(``PnP=False``: the reference's l1 ``Z_Update`` call uses an undefined ``lam``, ``:208``), and
``Unrolled_ADMM`` is inference-only: in training mode its forward raises under autograd when a
parameter requires grad (the engine writes through raw pointers, so no graph would reach ``self.Z`` /
``self.init``; the differentiable variant is ``UnrolledADMMGaussian``, whose X update has a HIP
backward); in eval mode it runs under ``torch.no_grad()`` and returns an output without a graph (only
parameter gradients can be dropped that way: an input ``y`` / ``kernel`` / ``alpha`` that requires grad raises).
"""
import warnings

import torch
import torch.nn as nn

from . import engine
from .nets import SubNet, XDenseUNet, ZUpdateResUNet, ZUpdateXDenseUNet


CONCURRENT_INIT_PIXELS = 1 << 23  # batch pixels from which the Gaussian init overlaps the SubNet


class Unrolled_ADMM(nn.Module):
    def __init__(self, n_iters=8, llh="Poisson", denoiser="ResUNet", PnP=True, subnet=True):
        super().__init__()
        if not PnP:
            raise NotImplementedError("PnP=False (l1 Z_Update) is broken in the reference (undefined lam)")
        if llh not in ("Poisson", "Gaussian"):
            raise ValueError("llh must be 'Poisson' or 'Gaussian'")
        self.n = n_iters
        self.llh = llh
        self.PnP = PnP
        self.subnet = subnet
        self.denoiser = denoiser
        # models/Unrolled_ADMM.py:163: the ResUNet for 'ResUNet', the XDenseUNet for anything else
        self.Z = ZUpdateResUNet() if denoiser == "ResUNet" else ZUpdateXDenseUNet()
        if self.subnet:
            self.init = SubNet(self.n)
        else:
            self.rho1_iters = nn.Parameter(torch.ones(size=[self.n]), requires_grad=True)
            self.rho2_iters = nn.Parameter(torch.ones(size=[self.n]), requires_grad=True)

    def rhos(self, kernel, alpha):
        if self.subnet:
            return self.init(kernel, alpha)
        return self.rho1_iters, self.rho2_iters

    def forward(self, y, kernel, alpha):
        if torch.is_grad_enabled() and any(torch.is_tensor(t) and t.requires_grad for t in (y, kernel, alpha)):
            # the reference's output is differentiable w.r.t. its inputs; the engine's is not: refuse rather
            # than return an output without the graph the caller asked for
            raise NotImplementedError(
                "Unrolled_ADMM on the HIP engine is inference-only: an input requires grad (detach it or call "
                "under torch.no_grad()); UnrolledADMMGaussian's X update has a HIP backward")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            if self.training:
                raise NotImplementedError(
                    "Unrolled_ADMM on the HIP engine is inference-only (call .eval(), wrap the call in "
                    "torch.no_grad() or freeze the parameters); train UnrolledADMMGaussian, whose X update "
                    "has a HIP backward")
            # eval mode with grad enabled (e.g. figures/grid_plot.ipynb calls the model and .detach()es):
            # the output carries no graph, as documented above
            if not Unrolled_ADMM._warned_grad:
                Unrolled_ADMM._warned_grad = True
                warnings.warn("Unrolled_ADMM (HIP engine) runs inference under torch.no_grad(): the output "
                              "does not require grad", stacklevel=2)
            with torch.no_grad():
                return self._forward(y, kernel, alpha)
        return self._forward(y, kernel, alpha)

    _warned_grad = False

    def _forward(self, y, kernel, alpha):
        N = y.shape[0]
        n = self.n
        if n == 0:
            st = engine.ADMMState(y, kernel, alpha, self.llh)
            with torch.no_grad():
                zero = torch.zeros(1, device=y.device)
                st.init((zero, 0))
            return st.zin * st.alpha.view(-1, 1, 1, 1) if self.llh == "Poisson" else st.zin
        st = engine.ADMMState(y, kernel, alpha, self.llh)
        rhos = None
        if self.subnet and "rhos" not in self.__dict__ and not st.init_reads_rho:
            # Gaussian: the init reads no rho.  Small stamps / batches (configs[1]): the SubNet and the init
            # in ONE launch whose workgroups share the CUs (gd_admm_init_subnet)
            packs = self.init.engine_packs(kernel)
            if packs is not None:
                rhos = st.init_with_subnet(*packs, self.init.n_out)
        if rhos is not None:
            rho1_iters, rho2_iters = self.init.split_rhos(rhos)
            done = True
        else:
            # large batches: the init on a side stream while the SubNet computes the rhos (4096 x 256^2: the
            # 0.4 ms SubNet hides behind the 1.4 ms init); below that a cross-queue join (~10 us) costs more
            # than it hides (256 x 48^2 kernel trace: a hipGraph replay started the SubNet only once the
            # 12 us init had drained)
            done = self.subnet and not st.init_reads_rho and N * st.H * st.W >= CONCURRENT_INIT_PIXELS
            if done:
                st.init_concurrent()
            try:
                rho1_iters, rho2_iters = self.rhos(kernel, alpha)
            except BaseException:
                # the side-stream init may still be writing st's buffers, which were allocated on the main
                # stream: join before they return to its pool
                st.join()
                raise
        r1 = engine.RhoSchedule(rho1_iters, N, st.dev)   # (pointer, stride) per iteration, computed once
        r2 = engine.RhoSchedule(rho2_iters, N, st.dev)
        if not done:
            st.init(r2[0])
        out = torch.empty_like(st.y)
        for it in range(n):
            z = self.Z(st.zin)
            st.step(z, r1[it], r2[it], r2[it + 1] if it + 1 < n else None, out=out)
        return out


class Wiener(nn.Module):
    def forward(self, y, psf, alpha):
        return engine.wiener(y, psf, alpha)


class Richard_Lucy(nn.Module):
    def __init__(self, n_iters):
        super().__init__()
        self.n_iters = n_iters

    def forward(self, y, psf):
        return engine.richardson_lucy(y, psf, self.n_iters)


class XUpdateGaussian(nn.Module):
    """models/unrolled_admm_gaussian.py:85-93 on the engine; the spectral constants (Y Ht, HtH) live
    in the forward's ``GaussXState`` instead of being passed as full spectra."""

    def forward(self, st, z, u, rho):
        return engine.gx_x_update(st, z, u, rho)


class UnrolledADMMGaussian(nn.Module):
    """models/unrolled_admm_gaussian.py:96-152.  Same constructor, attributes and state_dict keys
    (``Z.net.*`` with ResUNet nc=[32, 64, 128, 256], ``init.*`` SubNet with n outputs, or
    ``rho_iters``).  Under ``torch.no_grad`` the X update, the previous iteration's dual update and the
    next denoiser input ``rho x + u`` run fused in one engine call; with autograd on, the X update is
    a custom Function with the engine's backward and the elementwise updates are PyTorch ops."""

    def __init__(self, n_iters=8, denoiser="ResUNet", PnP=True, subnet=True, analysis=False):
        super().__init__()
        self.n_iters = n_iters
        self.denoiser = denoiser
        self.PnP = PnP
        self.subnet = subnet
        self.analysis = analysis
        self.X = XUpdateGaussian()
        self.Z = ZUpdateResUNet(nc=(32, 64, 128, 256))
        if self.subnet:
            self.init = SubNet(self.n_iters, n_out=self.n_iters, shift=True)
        else:
            self.rho_iters = nn.Parameter(torch.ones(size=[self.n_iters]), requires_grad=True)

    def forward(self, y, kernel, alpha):
        st = engine.GaussXState(y, kernel, alpha)       # max(y, 0) is applied on the device
        rho_iters = self.init(kernel, alpha) if self.subnet else None
        z = st.init()
        u = torch.zeros_like(st.y)
        x_list, z_list, u_list, rho_list = [], [], [], []
        fused = not torch.is_grad_enabled() and not self.analysis
        x, rho_prev = None, None
        for i in range(self.n_iters):
            rho = rho_iters[:, :, :, i].view(-1, 1, 1, 1) if self.subnet else self.rho_iters[i]
            if fused:
                x, zin, _ = st.x_update(z, u, rho, x_prev=x, rho_prev=rho_prev, zin=True)
                z = self.Z(zin)
                rho_prev = rho
            else:
                x = self.X(st, z, u, rho)
                z = self.Z(rho * x + u)
                u = u + rho * (x - z)
                x_list.append(x)
                z_list.append(z)
                u_list.append(u)
                rho_list.append(rho)
        if self.analysis:
            return x_list, z_list, u_list, rho_list
        return z


def laplacian_kernel():
    """utils/utils_torch.py:95-99: the 3x3 Laplacian stencil [1,1,3,3]."""
    return torch.tensor([[[[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]]]])


def placed_filter(ker, H, W, device):
    """The image ``psf_to_otf(ker, [1,1,H,W])[0]`` builds (utils/utils_torch.py:79-92), INCLUDING its
    behaviour for an odd 3x3 kernel: with ``center = 2`` the quadrant copies broadcast the 1-wide
    slices ``ker[2:, 2:]``, ``ker[2:, :2]``, ``ker[:2, 2:]`` over 2x2 blocks, so the Laplacian the
    reference regularises with is NOT the centred stencil.  Constant, built once per size (plumbing)."""
    k = ker.reshape(ker.shape[-2], ker.shape[-1]).float()
    img = torch.zeros(H, W)
    c = (k.shape[0] + 1) // 2
    img[:c, :c] = k[c:, c:]
    img[:c, -c:] = k[c:, :c]
    img[-c:, :c] = k[:c, c:]
    img[-c:, -c:] = k[:c, :c]
    return img.view(1, 1, H, W).to(device)


class Tikhonov(nn.Module):
    """models/Tikhonet.py:8-31: x = Re IFFT2(conj(H) FFT2(y/alpha) / (|H|^2 + lam [|L|^2])).  The
    Laplacian's |L|^2 is computed on the device once per (size, device) by direct DFT in double over
    its 7 taps (gd_filter_power_taps) and cached."""

    def __init__(self, filter="Identity"):
        super().__init__()
        if filter not in ("Identity", "Laplacian"):
            raise ValueError("filter must be 'Identity' or 'Laplacian'")
        self.filter = filter
        if self.filter == "Laplacian":
            self.lap = laplacian_kernel()
        self._ltl = {}

    def ltl(self, H, W, device):
        key = (H, W, str(device))
        if key not in self._ltl:
            self._ltl[key] = engine.filter_power_taps(placed_filter(self.lap, H, W, "cpu"), device)
        return self._ltl[key]

    def forward(self, y, psf, alpha, lam):
        ltl = self.ltl(y.shape[-2], y.shape[-1], y.device) if self.filter == "Laplacian" else None
        if not torch.is_tensor(lam):
            lam = torch.tensor(float(lam))
        return engine.tikhonov(y, psf, alpha, lam.to(y.device), ltl)


class Tikhonet(nn.Module):
    """models/Tikhonet.py:34-47: max(y, 0) -> Tikhonov(lam) -> XDenseUNet -> times alpha.  ``lam`` is
    a plain tensor as in the reference (not a Parameter, not in the state_dict)."""

    def __init__(self, filter="Identity"):
        super().__init__()
        self.tikhonov = Tikhonov(filter=filter)
        self.denoiser = XDenseUNet()
        self.lam = torch.tensor(1.0, requires_grad=True)

    def forward(self, y, psf, alpha):
        y = torch.clamp_min(y, 0.0)
        x = self.tikhonov(y, psf, alpha, self.lam)
        x = self.denoiser(x)
        return x * alpha


__all__ = ["Unrolled_ADMM", "UnrolledADMMGaussian", "XUpdateGaussian", "Wiener", "Richard_Lucy", "Tikhonov",
           "Tikhonet", "laplacian_kernel"]

"""Drop-in ``nn.Module``s with the reference's API, running the spectral path on the HIP engine.

* ``Unrolled_ADMM(n_iters=8, llh='Poisson', denoiser='ResUNet', PnP=True, subnet=True)`` -
  same constructor, attributes and ``state_dict`` keys as ``models/Unrolled_ADMM.py:153-215``
  (98 keys with the SubNet; ``rho1_iters``/``rho2_iters`` parameters with ``subnet=False``), same
  ``forward(y, kernel, alpha)`` semantics.  The ResUNet denoiser (``self.Z``) and the SubNet
  (``self.init``) stay in PyTorch; every spectral step goes through ``gdeconv.engine``.
* ``Wiener().forward(y, psf, alpha)`` - ``models/Wiener.py:10-20``.
* ``Richard_Lucy(n_iters).forward(y, psf)`` - ``models/Richard_Lucy.py:10-24``.

Differences from the reference, all deliberate: the device is taken from the input (the reference
hard-codes ``cuda:0``, ``models/Unrolled_ADMM.py:178``), the OTF is computed on the device (the
reference builds it on the CPU every forward, ``utils/utils_torch.py:81``), CPU tensors are
rejected (no CPU path), and unsupported reference variants raise instead of misbehaving:
``denoiser='XDenseUNet'`` (not on the hot path), ``PnP=False`` (the reference's l1 ``Z_Update``
call uses an undefined ``lam``, ``:208``).
"""
import torch
import torch.nn as nn

from . import engine
from .nets import SubNet, ZUpdateResUNet


def _rho_view(rho_iters, n, N):
    """(tensor, stride) for iteration n of a [N,1,1,n] SubNet output or an [n] parameter."""
    if rho_iters.dim() == 4:
        col = rho_iters[:, 0, 0, n]
        if col.dtype != torch.float32:
            col = col.float().contiguous()
        return col, (col.stride(0) if col.shape[0] == N and N > 1 else 0)
    t = rho_iters[n:n + 1]
    if t.dtype != torch.float32:
        t = t.float().contiguous()
    return t, 0


class Unrolled_ADMM(nn.Module):
    def __init__(self, n_iters=8, llh="Poisson", denoiser="ResUNet", PnP=True, subnet=True):
        super().__init__()
        if denoiser != "ResUNet":
            raise NotImplementedError("only denoiser='ResUNet' is on the accelerated path")
        if not PnP:
            raise NotImplementedError("PnP=False (l1 Z_Update) is broken in the reference (undefined lam)")
        if llh not in ("Poisson", "Gaussian"):
            raise ValueError("llh must be 'Poisson' or 'Gaussian'")
        self.n = n_iters
        self.llh = llh
        self.PnP = PnP
        self.subnet = subnet
        self.denoiser = denoiser
        self.Z = ZUpdateResUNet()
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
        N = y.shape[0]
        rho1_iters, rho2_iters = self.rhos(kernel, alpha)
        st = engine.ADMMState(y, kernel, alpha, self.llh)
        n = self.n
        if n == 0:
            with torch.no_grad():
                zero = torch.zeros(1, device=y.device)
                st.init((zero, 0))
            return st.zin * st.alpha.view(-1, 1, 1, 1) if self.llh == "Poisson" else st.zin
        st.init(_rho_view(rho2_iters, 0, N))
        out = torch.empty_like(st.y)
        for it in range(n):
            z = self.Z(st.zin)
            nxt = _rho_view(rho2_iters, it + 1, N) if it + 1 < n else None
            st.step(z, _rho_view(rho1_iters, it, N), _rho_view(rho2_iters, it, N), nxt, out=out)
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


__all__ = ["Unrolled_ADMM", "Wiener", "Richard_Lucy"]

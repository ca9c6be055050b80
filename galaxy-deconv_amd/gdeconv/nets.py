"""Host-side networks of the unrolled ADMM: the ResUNet denoiser (Z step) and the rho-predicting SubNet.

These stay in PyTorch-ROCm (MIOpen fp32 convolutions) per the north star; only the spectral ADMM
path is HIP.  The module *trees* are laid out so that ``state_dict`` keys are identical to the
reference checkpoints (98 keys for ``Unrolled_ADMM``):

* ``ResUNet``   mirrors ``models/ResUNet.py:7-42`` + ``models/resnet_basicblock.py:21-87``
  (head conv, 3 x [2 ResBlocks + 2x2 stride conv], body 2 ResBlocks, 3 x [2x2 conv-transpose +
  2 ResBlocks], tail conv; no bias, no norm; replicate-pad to a multiple of 8, additive skips).
* ``SubNet``    mirrors ``models/Unrolled_ADMM.py:59-90`` (|FFT(pad128(psf))|^2 -> 4 x
  [maxpool + 2 x (conv3x3+BN+ReLU)] -> MLP(1025, 64, 64, 2n) -> Softplus + 1e-6).

Key layout notes (the reference builds these with a ``sequential`` helper that flattens nested
Sequentials and returns a bare module for a single element):
  m_head / m_tail            -> bare Conv2d                         (keys ``m_head.weight``)
  m_downK                    -> Sequential(ResBlock, ResBlock, Conv2d(k2,s2))  (``m_down1.2.weight``)
  m_body                     -> Sequential(ResBlock, ResBlock)
  m_upK                      -> Sequential(ConvTranspose2d(k2,s2), ResBlock, ResBlock)
  ResBlock.res               -> Sequential(Conv2d, ReLU, Conv2d)    (``res.0.weight``, ``res.2.weight``)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class ResBlock(nn.Module):
    """x + conv(relu(conv(x))), 3x3, no bias (``resnet_basicblock.py:47-59`` with mode 'CRC')."""

    def __init__(self, channels):
        super().__init__()
        self.res = nn.Sequential(
            nn.Conv2d(channels, channels, 3, 1, 1, bias=False),
            nn.ReLU(inplace=True),
            nn.Conv2d(channels, channels, 3, 1, 1, bias=False),
        )

    def forward(self, x):
        return x + self.res(x)


def _down(cin, cout, nb):
    return nn.Sequential(*[ResBlock(cin) for _ in range(nb)],
                         nn.Conv2d(cin, cout, 2, 2, 0, bias=False))


def _up(cin, cout, nb):
    return nn.Sequential(nn.ConvTranspose2d(cin, cout, 2, 2, 0, bias=False),
                         *[ResBlock(cout) for _ in range(nb)])


class ResUNet(nn.Module):
    """4-level residual U-Net denoiser (``models/ResUNet.py:7-42``)."""

    def __init__(self, in_nc=1, out_nc=1, nc=(64, 128, 256, 512), nb=2):
        super().__init__()
        self.m_head = nn.Conv2d(in_nc, nc[0], 3, 1, 1, bias=False)
        self.m_down1 = _down(nc[0], nc[1], nb)
        self.m_down2 = _down(nc[1], nc[2], nb)
        self.m_down3 = _down(nc[2], nc[3], nb)
        self.m_body = nn.Sequential(*[ResBlock(nc[3]) for _ in range(nb)])
        self.m_up3 = _up(nc[3], nc[2], nb)
        self.m_up2 = _up(nc[2], nc[1], nb)
        self.m_up1 = _up(nc[1], nc[0], nb)
        self.m_tail = nn.Conv2d(nc[0], out_nc, 3, 1, 1, bias=False)
        # NHWC activations on the GPU: MIOpen's fp32 NHWC convolutions run the denoiser ~11 % faster
        # than NCHW on MI355X (tools/e2e_sweep.py: 89.8 -> 99.7 gal/s end to end at 256^2); same
        # arithmetic type (fp32), no TF32.  The parameters keep their values (state_dict unchanged).
        self.channels_last = True

    def forward(self, x):
        if self.channels_last and x.is_cuda:
            if not self.m_body[0].res[0].weight.is_contiguous(memory_format=torch.channels_last):
                self.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
            return self._forward(x).contiguous()
        return self._forward(x)

    def _forward(self, x):
        h, w = x.shape[-2:]
        pb, pr = (-h) % 8, (-w) % 8
        if pb or pr:
            x = F.pad(x, (0, pr, 0, pb), mode="replicate")
        x1 = self.m_head(x)
        x2 = self.m_down1(x1)
        x3 = self.m_down2(x2)
        x4 = self.m_down3(x3)
        x = self.m_body(x4)
        x = self.m_up3(x + x4)
        x = self.m_up2(x + x3)
        x = self.m_up1(x + x2)
        x = self.m_tail(x + x1)
        return x[..., :h, :w]


class ZUpdateResUNet(nn.Module):
    """Z step: ``z = ResUNet((x + u1).float())`` (runtime ``Z_Update_ResUNet`` at
    ``models/Unrolled_ADMM.py:349-357``; ``nc=(32, 64, 128, 256)`` for ``ZUpdateResUNet`` of
    ``models/unrolled_admm_gaussian.py:74-82``).  The attribute is ``net`` so keys read ``Z.net.*``."""

    def __init__(self, nc=(64, 128, 256, 512)):
        super().__init__()
        self.net = ResUNet(nc=tuple(nc))
        # galaxies per denoiser call: the ResUNet's activations are ~80 MB per 256^2 galaxy, so the
        # 4096-galaxy batch of configs[2] (~330 GB) must be micro-batched (hard parts).
        # None = auto: 2^25 pixels per call (512 galaxies at 256^2, ~40 GB).
        self.micro_batch = None

    def forward(self, z):
        z = z.float()
        N = z.shape[0]
        mb = self.micro_batch or max(1, (1 << 25) // max(1, z.shape[-1] * z.shape[-2]))
        if N <= mb:
            return self.net(z)
        if torch.is_grad_enabled():
            return torch.cat([self.net(z[i:i + mb]) for i in range(0, N, mb)])
        out = torch.empty_like(z)
        for i in range(0, N, mb):
            out[i:i + mb] = self.net(z[i:i + mb])
        return out


class ZUpdateXDenseUNet(ZUpdateResUNet):
    """Z step with the XDenseUNet denoiser: ``z = XDenseUNet(z.float())`` (``Z_Update_XDenseUNet``,
    ``models/Unrolled_ADMM.py:142-151``, selected by ``denoiser != 'ResUNet'`` at :163).  Keys read
    ``Z.net.*`` like the reference's; micro-batched like the ResUNet step."""

    def __init__(self):
        nn.Module.__init__(self)
        self.net = XDenseUNet()
        self.micro_batch = None


def _fold_conv_bn(conv, bn):
    """Eval-mode BatchNorm folded into the preceding conv: W' = W s, b' = (b - mean) s + beta,
    s = gamma / sqrt(var + eps).  Same function as conv -> BN up to fp32 rounding; it removes the
    BN pass (MIOpen's inference BN cost 1.4 ms per layer at N=4096 on the GPU)."""
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    w = conv.weight * s.view(-1, 1, 1, 1)
    b = (conv.bias - bn.running_mean) * s + bn.bias
    return w.contiguous(), b.contiguous()


class _DoubleConv(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.double_conv = nn.Sequential(
            nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
            nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))
        self._folded = None  # (key, [(w, b), (w, b)]) - not part of the state_dict
        self.fold_bn = True   # False: conv -> BN -> ReLU in the reference's op order

    def _fold_key(self):
        ts = [t for m in self.double_conv for t in list(m.parameters()) + list(m.buffers())]
        return tuple((t.data_ptr(), t._version) for t in ts)

    def forward(self, x):
        if self.training or not self.fold_bn:
            return self.double_conv(x)
        key = self._fold_key()
        if self._folded is None or self._folded[0] != key:
            with torch.no_grad():
                c1, b1, _, c2, b2, _ = self.double_conv
                self._folded = (key, [_fold_conv_bn(c1, b1), _fold_conv_bn(c2, b2)])
        (w1, bb1), (w2, bb2) = self._folded[1]
        x = F.relu(F.conv2d(x, w1, bb1, padding=1))
        return F.relu(F.conv2d(x, w2, bb2, padding=1))


class _Down(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), _DoubleConv(cin, cout))

    def forward(self, x):
        return self.maxpool_conv(x)


class SubNet(nn.Module):
    """Per-galaxy ADMM penalty predictor (``models/Unrolled_ADMM.py:59-90``).

    ``forward(kernel [N,1,h,w], alpha [N,1,1,1]) -> (rho1 [N,1,1,n], rho2 [N,1,1,n])``.
    The PSF is zero-padded (or cropped, for h > 128) to 128x128 with floor/ceil split, exactly as
    ``F.pad`` does at ``:79-81``.  In eval mode on ROCm the whole SubNet runs on the engine for a PSF
    of any shape (``_engine_kernel``); the torch.fft path below serves training and CPU tensors.
    """

    def __init__(self, n, n_out=None, shift=False):
        """``n_out`` MLP outputs (default 2n: rho1 and rho2 per iteration; n for the single rho of
        ``models/unrolled_admm_gaussian.py:43-71``, which returns [N,1,1,n]); ``shift``: that
        variant's ``fft2(ifftshift(k_pad))`` in the PyTorch path (|.|^2 is shift invariant)."""
        super().__init__()
        self.n = n
        self.n_out = 2 * n if n_out is None else n_out
        self.shift = shift
        self.conv_layers = nn.Sequential(_Down(1, 4), _Down(4, 8), _Down(8, 16), _Down(16, 16))
        self.use_engine = True  # ROCm + eval: fused HIP feature extractor (gd_subnet_features)
        self.mlp = nn.Sequential(nn.Linear(16 * 8 * 8 + 1, 64), nn.ReLU(inplace=True),
                                 nn.Linear(64, 64), nn.ReLU(inplace=True),
                                 nn.Linear(64, self.n_out), nn.Softplus())

    def _module_ids(self):
        """ids of every module object the engine packs read (the 4 _DoubleConvs, their conv / BN children,
        the 3 Linear layers): a child replaced in place (``net.mlp[0] = nn.Linear(...)``) changes the key."""
        ids = [id(self.conv_layers), id(self.mlp)]
        for down in self.conv_layers._modules.values():
            dc = down._modules["maxpool_conv"]._modules["1"]
            seq = dc._modules["double_conv"]._modules
            ids += (id(dc), id(seq["0"]), id(seq["1"]), id(seq["3"]), id(seq["4"]))
        m = self.mlp._modules
        ids += (id(m["0"]), id(m["2"]), id(m["4"]))
        return tuple(ids)

    def _pack_modules(self):
        """(conv/BN pairs, the 3 Linear layers, the 4 _DoubleConvs), looked up again whenever one of those
        module objects was replaced."""
        ident = self._module_ids()
        c = self.__dict__.get("_pmods")
        if c is None or c[0] != ident:
            dcs = [down.maxpool_conv[1] for down in self.conv_layers]
            pairs = []
            for dc in dcs:
                c1, b1, _, c2, b2, _ = dc.double_conv
                pairs += [(c1, b1), (c2, b2)]
            c = (ident, pairs, [self.mlp[0], self.mlp[2], self.mlp[4]], dcs)
            self.__dict__["_pmods"] = c
        return c[1], c[2], c[3]

    def _pack_key(self):
        """Data pointers and in-place versions of every tensor the engine packs (8 conv + BN, 3 Linear):
        changes on load_state_dict, .to(), optimizer steps.  ~15 us, against ~300 us for walking
        parameters() / buffers() of the module tree on every forward."""
        pairs, lins, _ = self._pack_modules()
        ts = []
        for c, b in pairs:
            p, q, r = c._parameters, b._parameters, b._buffers
            ts += (p["weight"], p["bias"], q["weight"], q["bias"], r["running_mean"], r["running_var"])
        for lin in lins:
            p = lin._parameters
            ts += (p["weight"], p["bias"])
        return tuple(map(torch.Tensor.data_ptr, ts)) + tuple([t._version for t in ts])

    def _engine_pack(self):
        """(conv pack, MLP pack) for the engine kernels, rebuilt only when a packed tensor changed.
        Conv pack: folded conv+BN weights of the 8 convs in gd_subnet_features order, per layer w then b,
        w tap-major ``[cin][3][3][cout]`` (include/gdeconv.h).  MLP pack: W1^T | b1 | W2^T | b2 | W3^T |
        b3 (transposed nn.Linear weights) for gd_subnet_rhos."""
        key = self._pack_key()
        c = self.__dict__.get("_epack")
        if c is None or c[0] != key:
            pairs, lins, _ = self._pack_modules()
            with torch.no_grad():
                parts = []
                for conv, bn in pairs:
                    w, b = _fold_conv_bn(conv, bn)
                    parts += [w.permute(1, 2, 3, 0).reshape(-1), b.reshape(-1)]
                conv_pack = torch.cat(parts).float().contiguous()
                parts = []
                for m in lins:
                    parts += [m.weight.t().reshape(-1), m.bias.reshape(-1)]
                mlp_pack = torch.cat(parts).float().contiguous()
            c = (key, conv_pack, mlp_pack)
            self.__dict__["_epack"] = c
        return c[1], c[2]

    def _packed_params(self):
        return self._engine_pack()[0]

    def _packed_mlp(self):
        return self._engine_pack()[1]

    def _double_convs(self):
        return self._pack_modules()[2]

    def _engine_ok(self, kernel):
        return (self.use_engine and kernel.is_cuda and not self.training
                and all(dc.fold_bn for dc in self._double_convs()))

    @staticmethod
    def _engine_kernel(kernel):
        """A PSF of any h x w -> an even square one of side <= 128 with the same |FFT2(pad128(.))|^2,
        which is all the SubNet sees (:79-83): sides above 128 cropped with F.pad's floor / ceil split
        (negative pads), then zeros appended below / right up to an even square side.  |FFT|^2 is
        invariant to the circular shift that separates any two placements of the same pixels in the
        128^2 grid, so the engine's psf_to_otf placement of the result gives the reference's feature
        map.  Even square PSFs of side <= 128 (every BASELINE config) pass through untouched."""
        h, w = kernel.shape[-2:]
        if h == w and h % 2 == 0 and h <= 128:
            return kernel
        if h > 128 or w > 128:
            t = -((128 - h) // 2) if h > 128 else 0   # -floor(0.5 (128 - h)): the rows F.pad removes on top
            l = -((128 - w) // 2) if w > 128 else 0   # noqa: E741
            kernel = kernel[..., t:t + min(h, 128), l:l + min(w, 128)]
            h, w = kernel.shape[-2:]
        s = max(h, w) + (max(h, w) & 1)
        return F.pad(kernel, (0, s - w, 0, s - h))

    def set_fold_bn(self, on):
        """Eval-mode BN folding (default on); off reproduces the reference's op order bit-exactly."""
        for m in self.modules():
            if isinstance(m, _DoubleConv):
                m.fold_bn = bool(on)
        return self

    def engine_packs(self, kernel):
        """(conv pack, MLP pack) on the kernel's device when this call can run the whole SubNet on the
        engine from the PSFs (eval, ROCm, even square PSF of side <= 64, MLP of <= 64 outputs and no
        autograd into it) - what ``Unrolled_ADMM`` hands to ``ADMMState.init_with_subnet``; else None."""
        from . import engine
        h, w = kernel.shape[-2:]
        if (not self._engine_ok(kernel) or h != w or h % 2 or h > 64
                or not engine.mlp_supported(self.n_out)):
            return None
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.mlp.parameters()):
            return None
        cpack, mpack = self._engine_pack()
        if cpack.device != kernel.device:
            cpack, mpack = cpack.to(kernel.device), mpack.to(kernel.device)
        return cpack, mpack

    def split_rhos(self, out):
        """[N, n_out] MLP output -> the forward's return value (rho1, rho2 halves, or the single rho)."""
        N = out.shape[0]
        out = out.view(N, 1, self.n_out)
        if self.n_out == self.n:
            return out.view(N, 1, 1, self.n)
        return out[:, :, 0:self.n].view(N, 1, 1, self.n), out[:, :, self.n:2 * self.n].view(N, 1, 1, self.n)

    def forward(self, kernel, alpha):
        N, _, h, w = kernel.shape
        if self._engine_ok(kernel):
            kernel = self._engine_kernel(kernel)
            h = kernel.shape[-1]
            # HIP path: OTF at 128^2 (|.|^2 is shift invariant, so equal to |FFT2(pad128)|^2), then the
            # conv stack (k_subnet_features) and one batched MLP launch (k_subnet_mlp: MLP, Softplus, + 1e-6)
            # (with autograd on and trainable MLP parameters - training UnrolledADMMGaussian, train.py:41 - the
            # MLP stays in PyTorch after k_subnet_features so its parameters get gradients)
            from . import engine
            dev = kernel.device
            cpack, mpack = self._engine_pack()
            if cpack.device != dev:
                cpack, mpack = cpack.to(dev), mpack.to(dev)
            mlp_ok = engine.mlp_supported(self.n_out)  # k_subnet_mlp: n_out <= 64 (kMaxOut)
            if mlp_ok and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.mlp.parameters())):
                if h <= 64:  # |FFT2(pad128(psf))|^2 inside the feature kernel (no OTF128 pre-pass)
                    out = engine.subnet_rhos_psf(kernel, cpack, mpack, alpha.reshape(-1), self.n_out)
                else:
                    out = engine.subnet_rhos(engine.psf_to_otf_half(kernel, N, 128, 128), cpack, mpack,
                                             alpha.reshape(-1), self.n_out)
                return self.split_rhos(out)
            feat = engine.subnet_features(engine.psf_to_otf_half(kernel, N, 128, 128), cpack)
        else:
            h1, h2 = (128 - h) // 2, 128 - h - (128 - h) // 2
            w1, w2 = (128 - w) // 2, 128 - w - (128 - w) // 2
            k_pad = F.pad(kernel, (w1, w2, h1, h2), "constant", 0)
            if self.shift:
                Hk = torch.fft.fft2(torch.fft.ifftshift(k_pad, dim=(-2, -1)))
            else:
                Hk = torch.fft.fftn(k_pad, dim=[2, 3])
            feat = self.conv_layers((torch.abs(Hk) ** 2).float())
        feat = torch.cat((feat.view(N, 1, 16 * 8 * 8), alpha.float().view(N, 1, 1)), dim=2)
        out = self.mlp(feat) + 1e-6
        if self.n_out == self.n:
            return out.view(N, 1, 1, self.n)
        rho1 = out[:, :, 0:self.n].view(N, 1, 1, self.n)
        rho2 = out[:, :, self.n:2 * self.n].view(N, 1, 1, self.n)
        return rho1, rho2


def count_params(m):
    return sum(p.numel() for p in m.parameters())


__all__ = ["ResUNet", "ResBlock", "ZUpdateResUNet", "SubNet", "count_params"]


# ---------------------------------------------------------------------------- Tikhonet denoiser
# XDenseUNet (``models/XDenseUNet.py``): a 3-level dense U-Net on 48x48 stamps, used by Tikhonet /
# ShapeNet after the Tikhonov solve.  PyTorch-ROCm (host side, not the spectral path).  Module tree
# laid out for the reference checkpoints' keys (``saved_models/Tikhonet_*_50epochs.pth``):
#   <block>.net.<i>.{0: BatchNorm2d, 2: SepConv.depthewise / .pointwise}   dense layers
#   Down: net.{0: BatchNorm2d, 2: Conv2d 1x1}   (then MaxPool2d(2))
#   Up:   net.{0: Conv2d 1x1 with bias}         (then nearest x2 upsampling)
class SepConv(nn.Module):
    """Depthwise k x k ('same' padding) then pointwise 1x1, no bias (``XDenseUNet.py:5-16``).
    The attribute name ``depthewise`` is the checkpoints' spelling."""

    def __init__(self, cin, cout, k=3):
        super().__init__()
        self.depthewise = nn.Conv2d(cin, cin, k, padding="same", groups=cin, bias=False)
        self.pointwise = nn.Conv2d(cin, cout, 1, bias=False)

    def forward(self, x):
        return self.pointwise(self.depthewise(x))


class DenseBlock(nn.Module):
    """``num_layers`` x [BN, ReLU, SepConv(c -> growth)], each output PREPENDED to the running stack
    (``torch.cat((out, y))``); ``skip`` prepends the block input once more (``XDenseUNet.py:19-41``)."""

    def __init__(self, num_layers, cin, growth=12, k=3, skip=False):
        super().__init__()
        self.skip_connection = skip
        self.net = nn.Sequential(*[
            nn.Sequential(nn.BatchNorm2d(cin + i * growth), nn.ReLU(inplace=True),
                          SepConv(cin + i * growth, growth, k))
            for i in range(num_layers)])

    def forward(self, x):
        y = x
        for layer in self.net:
            y = torch.cat((layer(y), y), dim=1)
        return torch.cat((x, y), dim=1) if self.skip_connection else y


class DenseDown(nn.Module):
    """BN, ReLU, 1x1 conv (no bias), 2x2 max-pool (``XDenseUNet.py:44-55``)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.net = nn.Sequential(nn.BatchNorm2d(cin), nn.ReLU(inplace=True),
                                 nn.Conv2d(cin, cout, 1, bias=False), nn.MaxPool2d(2, 2))

    def forward(self, x):
        return self.net(x)


class DenseUp(nn.Module):
    """1x1 conv with bias, nearest x2 upsampling (``XDenseUNet.py:58-67``)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.net = nn.Sequential(nn.Conv2d(cin, cout, 1, bias=True), nn.Upsample(scale_factor=(2, 2), mode="nearest"))

    def forward(self, x):
        return self.net(x)


class XDenseUNet(nn.Module):
    """``models/XDenseUNet.py:70-112``: channels 1 -> 112 (48^2) -> 220 (24^2) -> 352 (12^2) -> body
    at 6^2 -> 84 -> 72 -> 60 -> 1, skips by concatenation."""

    def __init__(self):
        super().__init__()
        self.input = nn.Sequential(nn.Conv2d(1, 32, 3, padding="same", bias=False), DenseBlock(4, 32, skip=True))
        self.down1 = nn.Sequential(DenseDown(112, 80), DenseBlock(5, 80, skip=True))
        self.down2 = nn.Sequential(DenseDown(220, 140), DenseBlock(6, 140, skip=True))
        self.body = nn.Sequential(DenseDown(352, 212), DenseBlock(7, 212), DenseUp(296, 84))
        self.up1 = nn.Sequential(DenseBlock(6, 436), DenseUp(508, 72))
        self.up2 = nn.Sequential(DenseBlock(5, 292), DenseUp(352, 60))
        self.output = nn.Sequential(DenseBlock(4, 172), nn.Conv2d(220, 1, 1, bias=True))

    def forward(self, x):
        x1 = self.input(x)
        x2 = self.down1(x1)
        x3 = self.down2(x2)
        x4 = self.body(x3)
        x5 = self.up1(torch.cat((x3, x4), dim=1))
        x6 = self.up2(torch.cat((x2, x5), dim=1))
        return self.output(torch.cat((x1, x6), dim=1))

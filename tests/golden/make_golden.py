"""Generate golden vectors by running the REFERENCE itself (read-only import) on CPU.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``models.Unrolled_ADMM`` / ``models.Wiener`` / ``models.Richard_Lucy`` /
``utils.utils_torch`` from /root/reference (torch CPU, fp32), loads the deterministic weights of
``gdeconv.weights.make_state_dict`` and writes small ``.npz`` fixtures next to this script.  Only
inputs and outputs are written - never reference source.  Per-iteration ADMM intermediates are
captured with forward hooks on the reference's ``V``/``Z``/``X`` sub-modules (the loop at
``models/Unrolled_ADMM.py:199-214`` is not modified).

Fixtures (all fp32; complex stored as [..., 2] real/imag):
  otf_conv.npz     G1  psf_to_otf + conv_fft_batch, tutorial 48^2 and seeded 256^2
  admm48.npz       G2  Unrolled_ADMM(n=2, 8; Gaussian, Poisson) at 48^2, N=2, with SubNet rhos
                       and per-iteration traces (v, z, x, zin); sample 0 = tutorial stamp
  admm256_id.npz   G3  Unrolled_ADMM(n=8) with denoiser = identity at 256^2, N=1, both llh
  wiener_rl.npz    G4  Wiener, Richard_Lucy(10), Richard_Lucy(100) at 48^2 (N=2) and 256^2 (N=1)
  admm256.npz      G5  Unrolled_ADMM(n=2, 8; Gaussian, Poisson) at 256^2, N=2 (seeded), real ResUNet/SubNet
                       with the generated weights: rhos, output and per-iteration traces (z, zin)
  state_dict_keys.json  the 98 keys + shapes of Unrolled_ADMM(n_iters=8)
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "galaxy-deconv_amd"))
sys.path.insert(0, REF)

from gdeconv.synth import make_batch           # noqa: E402
from gdeconv.weights import make_state_dict    # noqa: E402

# the drop-in's regular package ``models`` would shadow the reference's namespace package
sys.path[:] = [p for p in sys.path if os.path.abspath(p) != os.path.join(REPO, "galaxy-deconv_amd")]
for _m in [m for m in sys.modules if m == "models" or m.startswith("models.")]:
    del sys.modules[_m]
from models.Unrolled_ADMM import Unrolled_ADMM  # noqa: E402  (reference)
from models.Wiener import Wiener               # noqa: E402  (reference)
from models.Richard_Lucy import Richard_Lucy   # noqa: E402  (reference)
from utils.utils_torch import psf_to_otf, conv_fft_batch  # noqa: E402  (reference)

WEIGHT_SEED = 1234


def c2r(t):
    return torch.view_as_real(t.contiguous()).numpy().astype(np.float32)


def tutorial():
    load = lambda n: torch.load(os.path.join(REF, "tutorials", n + ".pth"), weights_only=True)  # noqa
    obs, psf = load("obs")[None, None], load("psf")[None, None]
    alpha = obs.mean().view(1, 1, 1, 1)
    return obs.float(), psf.float(), alpha.float()


def batch48():
    o0, p0, a0 = tutorial()
    o1, p1, a1, _ = make_batch(1, 48, seed=7)
    return torch.cat([o0, o1]), torch.cat([p0, p1]), torch.cat([a0, a1])


class Identity(torch.nn.Module):
    def forward(self, z):
        return z


def run_admm(obs, psf, alpha, n, llh, identity=False, trace=False):
    m = Unrolled_ADMM(n_iters=n, llh=llh, PnP=True, subnet=True)
    m.load_state_dict(make_state_dict(m, WEIGHT_SEED))
    m.eval()
    if identity:
        m.Z = Identity()
    rec = {"v": [], "z": [], "x": [], "zin": []}
    hooks = []
    if trace:
        def grab(*names):
            def hook(mod, inp, out):        # must return None (a value would replace the output)
                for nm, t in zip(names, (out, inp[0])):
                    rec[nm].append(t.clone())
            return hook
        hooks.append(m.V.register_forward_hook(grab("v")))
        hooks.append(m.Z.register_forward_hook(grab("z", "zin")))
        hooks.append(m.X.register_forward_hook(grab("x")))
    with torch.no_grad():
        rho1, rho2 = m.init(psf, alpha)
        out = m(obs, psf, alpha)
    for h in hooks:
        h.remove()
    res = {"out": out.numpy(), "rho1": rho1.numpy(), "rho2": rho2.numpy()}
    if trace:
        for k, v in rec.items():
            res[k] = torch.stack(v).numpy()       # [n, N, 1, H, W]
    return res


def main(only=None):
    """``only``: regenerate just that fixture ("otf_conv", "admm48", "admm256_id", "admm256", "wiener_rl"); the others are
    left as committed (their arrays are deterministic, but a rewrite changes the zip's timestamps)."""
    torch.manual_seed(0)
    torch.set_num_threads(8)
    want = (lambda name: only is None or only == name)

    # G1: psf_to_otf + conv_fft_batch
    o48, p48, a48 = tutorial()
    o256, p256, a256, _ = make_batch(1, 256, seed=11)
    g1 = {}
    for tag, (o, p) in {"48": (o48, p48), "256": (o256, p256)}.items():
        kpad, H = psf_to_otf(p, o.size())
        g1[f"obs{tag}"], g1[f"psf{tag}"] = o.numpy(), p.numpy()
        g1[f"kpad{tag}"] = kpad.numpy()
        g1[f"otf{tag}"] = c2r(H[..., : o.shape[-1] // 2 + 1])           # half spectrum
        g1[f"conv_H{tag}"] = conv_fft_batch(H, o).numpy()
        g1[f"conv_Ht{tag}"] = conv_fft_batch(torch.conj(H), o).numpy()
    if want("otf_conv"):
        np.savez_compressed(os.path.join(HERE, "otf_conv.npz"), **g1)

    # G2: ADMM at 48^2, N=2 (tutorial + seeded), real ResUNet/SubNet with generated weights
    obs, psf, alpha = batch48()
    g2 = {} if not want("admm48") else {"obs": obs.numpy(), "psf": psf.numpy(), "alpha": alpha.numpy()}
    for llh in ("Gaussian", "Poisson") if want("admm48") else ():
        for n in (2, 8):   # per-iteration traces for every (llh, n): Poisson is the reference's default llh
            r = run_admm(obs, psf, alpha, n, llh, trace=True)
            for k, v in r.items():
                g2[f"{llh}_n{n}_{k}"] = v
    if want("admm48"):
        np.savez_compressed(os.path.join(HERE, "admm48.npz"), **g2)

    # G3: ADMM spectral engine (denoiser = identity) at 256^2, N=1
    obs, psf, alpha, _ = make_batch(1, 256, seed=3)
    g3 = {"obs": obs.numpy(), "psf": psf.numpy(), "alpha": alpha.numpy()}
    for llh in ("Gaussian", "Poisson") if want("admm256_id") else ():
        r = run_admm(obs, psf, alpha, 8, llh, identity=True)
        for k, v in r.items():
            g3[f"{llh}_{k}"] = v
    if want("admm256_id"):
        np.savez_compressed(os.path.join(HERE, "admm256_id.npz"), **g3)

    # G5: ADMM at 256^2 (configs[2]'s stamp), N=2, the real ResUNet / SubNet with the generated weights:
    # per-iteration denoiser inputs (zin) and outputs (z) - z is the ResUNet's own tensor, never the buffer
    # the engine writes zin to, so a replay pins k_gal_reg / the Poisson two-pass on the product path.
    # v and x are not stored (not observable through the engine API; 256 KiB per galaxy-iteration each).
    if want("admm256"):
        obs, psf, alpha, _ = make_batch(2, 256, seed=256)
        g5 = {"obs": obs.numpy(), "psf": psf.numpy(), "alpha": alpha.numpy()}
        for llh in ("Gaussian", "Poisson"):
            for n in (2, 8):
                r = run_admm(obs, psf, alpha, n, llh, trace=True)
                for k in ("out", "rho1", "rho2", "z", "zin"):
                    g5[f"{llh}_n{n}_{k}"] = r[k]
        np.savez_compressed(os.path.join(HERE, "admm256.npz"), **g5)

    # G4: Wiener and Richardson-Lucy
    g4 = {}
    o1, p1, a1, _ = make_batch(1, 256, seed=5)
    for tag, (o, p, a) in ({"48": batch48(), "256": (o1, p1, a1)} if want("wiener_rl") else {}).items():
        g4[f"obs{tag}"], g4[f"psf{tag}"], g4[f"alpha{tag}"] = o.numpy(), p.numpy(), a.numpy()
        with torch.no_grad():
            g4[f"wiener{tag}"] = Wiener()(o, p, a).numpy()
            for n in (10, 100):
                g4[f"rl{n}_{tag}"] = Richard_Lucy(n)(o, p).numpy()
    if want("wiener_rl"):
        np.savez_compressed(os.path.join(HERE, "wiener_rl.npz"), **g4)

    m = Unrolled_ADMM(n_iters=8, llh="Gaussian")
    keys = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main(sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None)

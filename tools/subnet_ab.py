"""SubNet time per call: one fused launch per galaxy (k_subnet_rhos_psf) vs feature kernel + batched MLP
(gd_set_subnet_fused_max), at batches 256 / 1024 / 2048 / 4096 of 48 x 48 PSFs; rhos compared bitwise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "galaxy-deconv_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from gdeconv import _lib  # noqa: E402
from gdeconv.synth import make_batch  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
m = bench.build_model(8, "Gaussian", dev)
old = lib.gd_set_subnet_fused_max(-1)
for N in (256, 1024, 2048, 4096):
    _, psf, alpha, _ = make_batch(N, 48, seed=5, device=dev)
    res = {}
    for name, thr in (("two launches", 0), ("fused", 1 << 30)):
        lib.gd_set_subnet_fused_max(thr)
        lib.gd_profile_reset()
        with torch.no_grad():
            for _ in range(3):
                r = m.init(psf, alpha)
            torch.cuda.synchronize()
            _lib.profile_enable(2)
            for _ in range(20):
                r = m.init(psf, alpha)
            torch.cuda.synchronize()
            _lib.profile_enable(0)
        st = _lib.profile_collect()
        res[name] = (sum(ms / n for ms, n in st.values()) * 1e3, torch.cat([r[0].flatten(), r[1].flatten()]).cpu(),
                     {k: round(ms / n * 1e3, 1) for k, (ms, n) in st.items()})
    same = torch.equal(res["fused"][1], res["two launches"][1])
    print(f"N={N}: two launches {res['two launches'][0]:.1f} us {res['two launches'][2]}, "
          f"fused {res['fused'][0]:.1f} us {res['fused'][2]}; bit-identical {same}", flush=True)
lib.gd_set_subnet_fused_max(old)

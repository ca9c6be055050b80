import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "galaxy-deconv_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm device (MI355X) and the built HIP engine")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm device is visible")
    return torch.device("cuda:0")


TOL = 1e-5
# A galaxy may use the relaxed bound (2b) below only when the reference's own distance from the exact
# result is at least this fraction of tol: there the reference's rounding, not the engine's, decides
# whether engine-vs-reference crosses tol.
RELAX_MIN_FRAC = 0.5
# The cases that need it (engine-vs-reference above 1e-5 on some galaxy), as measured; every one of them is
# listed in README.md's Parity row.  A case outside this set that would need the relaxed bound fails.
RELAXED_CASES = ("Tikhonov(Laplacian, lam=2.0) 255x255",)


def parity_gate(tag, out, gold, ref64, tol=TOL):
    """The parity gate (normwise max|a - b| <= 1e-5 max|b| per galaxy), per galaxy:

      (1) engine vs the fp64 oracle <= tol (the engine's own error), and
      (2a) engine vs reference <= tol (the default: the reference's own golden vectors bind), or
      (2b) only for a galaxy whose reference-vs-fp64 error is itself >= RELAX_MIN_FRAC * tol, and only in a
           case listed in RELAXED_CASES: engine vs reference <= tol + that galaxy's reference-vs-fp64.

    (2b) exists because a deconvolution amplifies fp32 rounding where |H|^2 is small: for the ill-conditioned
    Tikhonov-Laplacian the reference's own fp32 output sits ~1.1e-5 from the exact result, and the engine
    (3.9e-7 from it) then sits as far from the reference as the reference sits from the exact answer.  The
    record (stdout, $GD_PARITY_LOG) names the galaxies that used (2b).  Returns the record."""
    import json

    import admm_oracle as O
    e64_g = O.normwise_error(out, ref64)
    eref_g = O.normwise_error(out, gold)
    r64_g = O.normwise_error(gold, ref64)
    relaxed = [int(i) for i in range(len(eref_g))
               if eref_g[i] > tol and r64_g[i] >= RELAX_MIN_FRAC * tol and eref_g[i] <= tol + r64_g[i]]
    e64, eref, r64 = float(e64_g.max()), float(eref_g.max()), float(r64_g.max())
    rec = {"case": tag, "engine_vs_fp64_normwise": e64, "engine_vs_reference_normwise": eref,
           "reference_vs_fp64_normwise": r64, "gate_engine_vs_reference": tol,
           "relaxed_galaxies": relaxed}
    print(f"[parity-gate] {tag}: engine-vs-fp64 {e64:.3e} (<= {tol:.0e}), engine-vs-reference {eref:.3e} "
          f"(<= {tol:.0e}; reference-vs-fp64 {r64:.3e}; relaxed galaxies {relaxed})")
    log = os.environ.get("GD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert e64 <= tol, rec
    assert not relaxed or tag in RELAXED_CASES, rec
    strict = [i for i in range(len(eref_g)) if i not in relaxed]
    assert not strict or float(eref_g[strict].max()) <= tol, rec
    return rec

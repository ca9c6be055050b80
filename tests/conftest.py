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


def parity_gate(tag, out, gold, ref64, tol=TOL):
    """The engine-limited parity gate (normwise max|a - b| <= 1e-5 max|b| per galaxy).

    A deconvolution amplifies fp32 rounding where |H|^2 is small, so for ill-conditioned cases (Tikhonov-
    Laplacian, Richardson-Lucy(100)) the reference's own fp32 output can sit close to 1e-5 from the exact
    result: a gate of engine-vs-reference <= 1e-5 alone would then flip on the REFERENCE's rounding.  Here
      (1) engine vs the fp64 oracle  <= tol                       (the engine's own error), and
      (2) engine vs reference        <= tol + reference vs fp64   (the triangle inequality's slack: the
          engine agrees with the reference as well as two results each within tol of the exact one can),
    both recorded (stdout, $GD_PARITY_LOG).  Returns the record."""
    import json

    import admm_oracle as O
    e64 = float(O.normwise_error(out, ref64).max())
    eref = float(O.normwise_error(out, gold).max())
    r64 = float(O.normwise_error(gold, ref64).max())
    rec = {"case": tag, "engine_vs_fp64_normwise": e64, "engine_vs_reference_normwise": eref,
           "reference_vs_fp64_normwise": r64, "gate_engine_vs_reference": tol + r64}
    print(f"[parity-gate] {tag}: engine-vs-fp64 {e64:.3e} (<= {tol:.0e}), engine-vs-reference {eref:.3e} "
          f"(<= {tol:.0e} + reference-vs-fp64 {r64:.3e})")
    log = os.environ.get("GD_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert e64 <= tol, rec
    assert eref <= tol + r64, rec
    return rec

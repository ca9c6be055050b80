"""Deterministic weights for ``Unrolled_ADMM`` (the reference's pretrained ADMM checkpoints are
absent: ``.MISSING_LARGE_BLOBS`` lists ``saved_models/Gaussian_PnP_ADMM_{2,4,8}iters_*.pth``).

``make_state_dict(model_or_keys, seed)`` draws every tensor from one numpy ``PCG64(seed)`` stream in
``state_dict`` key order, so the same seed gives bit-identical tensors for the reference module
(when golden vectors are generated in the build container) and for this framework's drop-in module
(on the GPU box).  The recipe is part of the fixture contract - changing it invalidates
``tests/golden``.

Recipe per key (shape S, fan = numel / S[0]):
  * conv / linear / conv-transpose weights : N(0,1) * gain / sqrt(fan)
      gain = 0.35 inside ResBlock residual branches (``.res.``), 1.0 elsewhere - keeps the random
      ResUNet's output at the scale of its input so unrolled ADMM stays well conditioned;
  * biases                                 : 0.05 * N(0,1)
  * BatchNorm weight / bias                : 1 + 0.1 N(0,1) / 0.1 N(0,1)
  * BatchNorm running_mean / running_var   : 0.1 N(0,1) / 1 + 0.2 |N(0,1)|
  * num_batches_tracked                    : 0
  * rho1_iters / rho2_iters (subnet=False) : 0.5 + U(0,1)
"""
import numpy as np
import torch


def _is_bn(key, shape, keys):
    # BatchNorm tensors are the 1-D weight/bias whose module also owns running_mean.
    mod = key.rsplit(".", 1)[0]
    return (mod + ".running_mean") in keys


def make_state_dict(template, seed=20250307):
    """Return an ordered dict of tensors with the keys/shapes/dtypes of ``template``.

    ``template`` is an ``nn.Module`` or a ``state_dict``-like mapping of key -> tensor."""
    sd = template.state_dict() if hasattr(template, "state_dict") else template
    keys = set(sd.keys())
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for key, ref in sd.items():
        shape = tuple(ref.shape)
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[key] = torch.zeros((), dtype=ref.dtype)
            continue
        n = int(np.prod(shape)) if shape else 1
        if leaf in ("rho1_iters", "rho2_iters"):
            val = 0.5 + rng.random(n)
        elif leaf == "running_mean":
            val = 0.1 * rng.standard_normal(n)
        elif leaf == "running_var":
            val = 1.0 + 0.2 * np.abs(rng.standard_normal(n))
        elif _is_bn(key, shape, keys):
            z = rng.standard_normal(n)
            val = (1.0 + 0.1 * z) if leaf == "weight" else 0.1 * z
        elif leaf == "bias":
            val = 0.05 * rng.standard_normal(n)
        else:
            fan = max(1, n // shape[0])
            gain = 0.35 if ".res." in key else 1.0
            val = rng.standard_normal(n) * (gain / np.sqrt(fan))
        out[key] = torch.from_numpy(val.astype(np.float32).reshape(shape)).to(ref.dtype)
    return out


__all__ = ["make_state_dict"]

"""Golden vectors for the dataset API, made by running the REFERENCE's own
``Galaxy_Dataset`` (utils/utils_data.py:44-103, read-only import) on a small seeded dataset folder
in the reference's layout:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ingest.py

ingest.npz holds the dataset's raw arrays (obs / psf / gt, fp32; written back to disk by the tests
with torch.save in the same layout) and what the reference's loader returns for every train and
test item: obs [1,H,W], psf [1,h,w], alpha [1,1,1] (= obs.ravel().mean()), gt [1,H,W].
Only inputs and outputs are written - never reference source.
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)
from utils.utils_data import Galaxy_Dataset, down_sample, get_flux  # noqa: E402  (reference)

N_TRAIN, N_TEST, H, h = 5, 3, 48, 48


def make_arrays(seed=2025):
    rng = np.random.default_rng(seed)
    n = N_TRAIN + N_TEST
    obs = (rng.normal(0.0, 19.04, (n, H, H)) + rng.uniform(0, 300, (n, 1, 1))).astype(np.float32)
    psf = rng.uniform(0, 1, (n, h, h)).astype(np.float32)
    psf /= 16 * psf.sum(axis=(1, 2), keepdims=True)
    gt = rng.uniform(0, 50, (n, H, H)).astype(np.float32)
    return obs, psf, gt


def write_folder(root, obs, psf, gt):
    """The reference's on-disk layout (generate_data.py writes the same names)."""
    n = obs.shape[0]
    for sub in ("psf", "obs", "gt"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    for i in range(n):
        torch.save(torch.from_numpy(psf[i].copy()), os.path.join(root, "psf", f"psf_{i}.pth"))
        torch.save(torch.from_numpy(obs[i].copy()), os.path.join(root, "obs", f"obs_{i}.pth"))
        torch.save(torch.from_numpy(gt[i].copy()), os.path.join(root, "gt", f"gt_{i}.pth"))
    info = {"n_total": n, "n_train": N_TRAIN, "n_test": n - N_TRAIN, "sequence": list(range(n))}
    with open(os.path.join(root, "info.json"), "w") as f:
        json.dump(info, f)


def main():
    obs, psf, gt = make_arrays()
    g = {"obs_raw": obs, "psf_raw": psf, "gt_raw": gt}
    with tempfile.TemporaryDirectory() as d:
        write_folder(d, obs, psf, gt)
        for train, tag in ((True, "train"), (False, "test")):
            ds = Galaxy_Dataset(data_path=d, train=train)
            items = [ds[i] for i in range(len(ds))]
            g[f"{tag}_obs"] = np.stack([it[0][0].numpy() for it in items])
            g[f"{tag}_psf"] = np.stack([it[0][1].numpy() for it in items])
            g[f"{tag}_alpha"] = np.stack([it[0][2].numpy() for it in items])
            g[f"{tag}_gt"] = np.stack([it[1].numpy() for it in items])
    # the module's two helpers (generate_data.py uses them): 4x box down-sampling, magnitude -> flux
    ds_in = np.random.default_rng(7).uniform(0, 1, (192, 192)).astype(np.float32)
    g["ds_in"], g["ds_out"] = ds_in, down_sample(torch.from_numpy(ds_in)).numpy()
    mags = np.array([20.0, 23.5, 25.2], np.float64)
    g["flux_mag"] = mags
    g["flux"] = np.array([get_flux(m, 30.0, 32.363, 4.5, 0.9) for m in mags], np.float64)
    np.savez_compressed(os.path.join(HERE, "ingest.npz"), **g)
    print({k: v.shape for k, v in g.items()})


if __name__ == "__main__":
    main()

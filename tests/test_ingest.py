"""Dataset API and packed ingest, on CPU: the reference-layout loader, the
GDPACK01 writer and the native reader (C ABI gd_pack_*, host-only) against the reference's own
Galaxy_Dataset outputs (tests/golden/ingest.npz, made by tests/golden/make_golden_ingest.py).
Bar: bit-exact (byte work and the reference's own alpha reduction)."""
import os

import numpy as np
import pytest
import torch

from conftest import golden

G = golden("ingest.npz")
N_TRAIN = G["train_obs"].shape[0]


def _write_folder(root):
    import json
    obs, psf, gt = G["obs_raw"], G["psf_raw"], G["gt_raw"]
    n = obs.shape[0]
    for sub in ("psf", "obs", "gt"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    for i in range(n):
        torch.save(torch.from_numpy(psf[i].copy()), os.path.join(root, "psf", f"psf_{i}.pth"))
        torch.save(torch.from_numpy(obs[i].copy()), os.path.join(root, "obs", f"obs_{i}.pth"))
        torch.save(torch.from_numpy(gt[i].copy()), os.path.join(root, "gt", f"gt_{i}.pth"))
    with open(os.path.join(root, "info.json"), "w") as f:
        json.dump({"n_total": n, "n_train": N_TRAIN, "n_test": n - N_TRAIN, "sequence": list(range(n))}, f)
    return root


@pytest.fixture(scope="module")
def folder(tmp_path_factory):
    return _write_folder(str(tmp_path_factory.mktemp("galaxies")))


@pytest.fixture(scope="module")
def packed(folder, tmp_path_factory):
    from gdeconv.ingest import pack_dataset
    return pack_dataset(folder, str(tmp_path_factory.mktemp("pack") / "ds.gdpack"))


def _check_items(items, tag):
    for k, ((obs, psf, alpha), gt) in enumerate(items):
        assert np.array_equal(obs.numpy(), G[f"{tag}_obs"][k])
        assert np.array_equal(psf.numpy(), G[f"{tag}_psf"][k])
        assert np.array_equal(alpha.numpy(), G[f"{tag}_alpha"][k])
        assert np.array_equal(gt.numpy(), G[f"{tag}_gt"][k])
        assert obs.shape == (1, 48, 48) and psf.shape == (1, 48, 48) and alpha.shape == (1, 1, 1)


@pytest.mark.parametrize("train,tag", [(True, "train"), (False, "test")])
def test_galaxy_dataset_matches_reference(folder, train, tag):
    from gdeconv.ingest import Galaxy_Dataset
    ds = Galaxy_Dataset(folder, train=train)
    assert len(ds) == G[f"{tag}_obs"].shape[0]
    _check_items([ds[i] for i in range(len(ds))], tag)


def test_galaxy_dataset_missing_info_is_empty(tmp_path):
    from gdeconv.ingest import Galaxy_Dataset
    assert len(Galaxy_Dataset(str(tmp_path))) == 0  # the reference logs and yields an empty dataset


def test_test_loader_batch_one(folder):
    from gdeconv.ingest import get_dataloader
    dl = get_dataloader(folder, train=False)
    (obs, psf, alpha), gt = next(iter(dl))
    assert obs.shape == (1, 1, 48, 48) and alpha.shape == (1, 1, 1, 1)
    assert np.array_equal(alpha.numpy()[0], G["test_alpha"][0])


@pytest.mark.parametrize("train,tag", [(True, "train"), (False, "test")])
def test_packed_dataset_matches_reference(packed, train, tag):
    from gdeconv.ingest import PackedGalaxies
    with PackedGalaxies(packed) as pk:
        assert (pk.n, pk.H, pk.W, pk.h, pk.w, pk.has_gt) == (8, 48, 48, 48, 48, 1)
        assert pk.info["n_train"] == N_TRAIN
        ds = pk.dataset(train)
        assert len(ds) == G[f"{tag}_obs"].shape[0]
        _check_items([ds[i] for i in range(len(ds))], tag)
        with pytest.raises(IndexError):
            ds[len(ds)]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_packed_ranges_and_gathers(packed, threads):
    from gdeconv.ingest import PackedGalaxies
    allobs = np.concatenate([G["train_obs"], G["test_obs"]])
    allalpha = np.concatenate([G["train_alpha"], G["test_alpha"]])
    with PackedGalaxies(packed, threads=threads) as pk:
        assert np.array_equal(pk.read("obs", 0, 8).numpy(), allobs)
        assert np.array_equal(pk.read("obs", 3, 4).numpy(), allobs[3:7])
        assert np.array_equal(pk.read("alpha", 0, 8).numpy(), allalpha)
        idx = [6, 1, 1, 7, 0]
        assert np.array_equal(pk.gather("obs", idx).numpy(), allobs[idx])
        assert np.array_equal(pk.gather("alpha", idx).numpy(), allalpha[idx])
        assert pk.read("psf", 2, 0).shape[0] == 0


def test_write_pack_from_arrays_matches_folder_pack(packed, tmp_path):
    from gdeconv.ingest import write_pack
    p2 = write_pack(str(tmp_path / "b.gdpack"), G["obs_raw"], G["psf_raw"], gt=G["gt_raw"],
                    info={"n_total": 8, "n_train": N_TRAIN, "n_test": 8 - N_TRAIN, "sequence": list(range(8))})
    assert open(p2, "rb").read() == open(packed, "rb").read()


def test_large_read_spans_many_blocks(tmp_path):
    """> 4 MiB per section: the reader splits it over its threads."""
    from gdeconv.ingest import PackedGalaxies, write_pack
    rng = np.random.default_rng(0)
    obs = rng.normal(size=(40, 256, 256)).astype(np.float32)  # 10 MiB
    psf = rng.uniform(size=(40, 48, 48)).astype(np.float32)
    p = write_pack(str(tmp_path / "big.gdpack"), obs, psf)
    with PackedGalaxies(p, threads=5) as pk:
        assert not pk.has_gt
        assert np.array_equal(pk.read("obs", 0, 40).numpy()[:, 0], obs)
        assert np.array_equal(pk.read("obs", 7, 21).numpy()[:, 0], obs[7:28])
        al = pk.read("alpha", 0, 40).numpy().reshape(-1)
        ref = np.array([torch.from_numpy(obs[i]).ravel().mean().float().item() for i in range(40)], np.float32)
        assert np.array_equal(al, ref)


def test_reader_errors(packed, tmp_path):
    from gdeconv._lib import EngineError
    from gdeconv.ingest import PackedGalaxies, write_pack
    with pytest.raises(EngineError, match="cannot open"):
        PackedGalaxies(str(tmp_path / "missing.gdpack"))
    bad = tmp_path / "bad.gdpack"
    bad.write_bytes(b"NOTAPACK" + bytes(8000))
    with pytest.raises(EngineError, match="not a GDPACK01"):
        PackedGalaxies(str(bad))
    trunc = tmp_path / "trunc.gdpack"
    trunc.write_bytes(open(packed, "rb").read()[:9000])
    with pytest.raises(EngineError, match="truncated"):
        PackedGalaxies(str(trunc))
    p = write_pack(str(tmp_path / "nogt.gdpack"), G["obs_raw"], G["psf_raw"])
    with PackedGalaxies(p) as pk:
        with pytest.raises(EngineError, match="out of bounds"):
            pk.read("obs", 5, 4)
        with pytest.raises(EngineError, match="no ground truth"):
            pk.read("gt", 0, 1)
        with pytest.raises(EngineError, match="out of bounds"):
            pk.gather("obs", [0, 8])


def test_utils_data_helpers_match_reference():
    from utils.utils_data import down_sample, get_flux
    assert np.array_equal(down_sample(torch.from_numpy(G["ds_in"])).numpy(), G["ds_out"])
    got = np.array([get_flux(m, 30.0, 32.363, 4.5, 0.9) for m in G["flux_mag"]])
    assert np.array_equal(got, G["flux"])

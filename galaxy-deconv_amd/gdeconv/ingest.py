"""Batched data ingest and the reference's dataset API.

* ``Galaxy_Dataset`` / ``get_dataloader`` mirror ``utils/utils_data.py:44-136``: the same folder
  layout (``info.json``, ``psf/psf_{i}.pth``, ``obs/obs_{i}.pth``, ``gt/gt_{i}.pth``), the same
  train/test split by ``n_train``, the same item ``((obs [1,H,W], psf [1,h,w], alpha [1,1,1]), gt)``
  with ``alpha = obs.ravel().mean()``.  Tensors are loaded with ``torch.load(weights_only=True)``.
* ``pack_dataset`` converts such a folder into ONE GDPACK01 file (format: ``csrc/gd_ingest.hpp``):
  contiguous fp32 sections obs / psf / gt / alpha + the info JSON, alpha precomputed exactly as the
  reference computes it.
* ``PackedGalaxies`` reads whole batches of a packed file through the native reader (C ABI
  ``gd_pack_*``: a pool of ``pread`` threads into pinned host memory; ctypes drops the GIL).
* ``DeviceBatches`` streams batches to the GPU: a reader thread fills pinned host slots ahead of
  use while the previous batch computes; each slot goes up on a dedicated copy stream (SDMA) and
  torch's current stream waits on its event, so the H2D copy of batch i overlaps the engine's work
  on batch i-1.  Batches come out in the drop-in's shapes: obs [B,1,H,W], psf [B,1,h,w],
  alpha [B,1,1,1] (+ gt [B,1,H,W]).
"""
import ctypes
import json
import logging
import os
import queue
import threading

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, random_split

from . import _lib

SECTIONS = {"obs": 0, "psf": 1, "gt": 2, "alpha": 3, "info": 4}
HEADER_BYTES = 4096
_ALIGN = 4096
_MAGIC = b"GDPACK01"


# ------------------------------------------------------------------ the reference's dataset API
def reference_alpha(obs):
    """``alpha = obs.ravel().mean().float()`` of one [1,H,W] (or [H,W]) observation, as
    ``utils/utils_data.py:100`` computes it (same op, same reduction order: bit-identical)."""
    return obs.ravel().mean().float()


class Galaxy_Dataset(Dataset):
    """``utils/utils_data.py:44-103``: per-file galaxy dataset (3 ``torch.load`` per item)."""

    def __init__(self, data_path, train=True, psf_folder="psf/", obs_folder="obs/", gt_folder="gt/"):
        super().__init__()
        self.logger = logging.getLogger("Dataset")
        self.data_path = data_path
        self.train = train
        self.psf_folder, self.obs_folder, self.gt_folder = psf_folder, obs_folder, gt_folder
        self.n_total, self.n_train, self.n_test = 0, 0, 0
        self.sequence = []
        self.info = {}
        self.info_file = os.path.join(self.data_path, "info.json")
        try:  # the reference logs and continues with an empty dataset (:71-80)
            with open(self.info_file, "r") as f:
                self.info = json.load(f)
            self.n_total = self.info["n_total"]
            self.n_train = self.info["n_train"]
            self.n_test = self.info["n_test"]
            self.sequence = self.info["sequence"]
        except Exception:
            self.logger.exception(" Failed reading information from %s.", self.info_file)

    def __len__(self):
        return self.n_train if self.train else self.n_test

    def load_item(self, idx):
        """Galaxy ``idx`` of the whole dataset (train and test share the index space)."""
        def ld(folder, stem):
            return torch.load(os.path.join(self.data_path, folder, f"{stem}_{idx}.pth"), weights_only=True)
        psf = ld(self.psf_folder, "psf").unsqueeze(0)
        obs = ld(self.obs_folder, "obs").unsqueeze(0)
        gt = ld(self.gt_folder, "gt").unsqueeze(0)
        alpha = torch.Tensor(reference_alpha(obs)).view(1, 1, 1)
        return (obs, psf, alpha), gt

    def __getitem__(self, i):
        return self.load_item(i if self.train else i + self.n_train)


def get_dataloader(data_path, train=True, train_val_split=0.8, batch_size=32, num_workers=18, pin_memory=True,
                   psf_folder="psf/", obs_folder="obs/", gt_folder="gt/"):
    """``utils/utils_data.py:106-136``: (train_loader, val_loader) or the batch-1 test_loader."""
    if train:
        ds = Galaxy_Dataset(data_path=data_path, train=True)
        n_tr = int(train_val_split * len(ds))
        tr, va = random_split(ds, [n_tr, len(ds) - n_tr])
        return (DataLoader(tr, batch_size=batch_size, shuffle=True, num_workers=num_workers, pin_memory=pin_memory),
                DataLoader(va, batch_size=batch_size, shuffle=False, num_workers=num_workers, pin_memory=pin_memory))
    ds = Galaxy_Dataset(data_path=data_path, train=False, psf_folder=psf_folder, obs_folder=obs_folder,
                        gt_folder=gt_folder)
    return DataLoader(ds, batch_size=1, shuffle=False)


# ------------------------------------------------------------------ GDPACK01 writer
def _f32(a):
    if torch.is_tensor(a):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=np.float32)


class PackWriter:
    """Streaming GDPACK01 writer: sections are pre-placed, galaxies written at their offsets."""

    def __init__(self, path, n, H, W, h, w, has_gt, info=None):
        self.path, self.n = path, int(n)
        self.shape = (H, W, h, w)
        self.has_gt = bool(has_gt)
        info_b = json.dumps(info or {}).encode()
        sizes = [n * H * W * 4, n * h * w * 4, n * H * W * 4 if has_gt else 0, n * 4, len(info_b)]
        offs, o = [], HEADER_BYTES
        for sz in sizes:
            offs.append(o)
            o += (sz + _ALIGN - 1) // _ALIGN * _ALIGN
        self.offsets, self.sizes = offs, sizes
        hdr = np.zeros(HEADER_BYTES, dtype=np.uint8)
        fixed = (_MAGIC + np.array([n], "<i8").tobytes() + np.array([H, W, h, w, int(has_gt), 0], "<i4").tobytes()
                 + np.array(offs, "<i8").tobytes() + np.array(sizes, "<i8").tobytes())
        hdr[:len(fixed)] = np.frombuffer(fixed, dtype=np.uint8)
        self.f = open(path, "wb")
        self.f.write(hdr.tobytes())
        self.f.truncate(o)
        self.f.seek(offs[4])
        self.f.write(info_b)

    def write(self, section, g0, arr):
        """Galaxies [g0, g0 + len(arr)) of a section (fp32, any leading shape)."""
        s = SECTIONS[section]
        a = _f32(arr)
        item = {0: self.shape[0] * self.shape[1], 1: self.shape[2] * self.shape[3],
                2: self.shape[0] * self.shape[1], 3: 1}[s]
        if a.size % item or g0 < 0 or g0 + a.size // item > self.n or (s == 2 and not self.has_gt):
            raise ValueError(f"bad {section} block for galaxies from {g0}")
        self.f.seek(self.offsets[s] + g0 * item * 4)
        self.f.write(a.tobytes())

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_pack(path, obs, psf, gt=None, alpha=None, info=None):
    """Pack in-memory batches: obs [n,(1,)H,W], psf [n,(1,)h,w], gt like obs; alpha defaults to the
    reference's per-galaxy ``obs.ravel().mean()``."""
    obs_t = obs if torch.is_tensor(obs) else torch.from_numpy(np.asarray(obs))
    obs_t = obs_t.detach().cpu().float()
    n, H, W = obs_t.shape[0], obs_t.shape[-2], obs_t.shape[-1]
    psf_a = _f32(psf)
    h, w = psf_a.shape[-2], psf_a.shape[-1]
    if alpha is None:
        alpha = np.array([float(reference_alpha(obs_t[i].reshape(1, H, W))) for i in range(n)], np.float32)
    with PackWriter(path, n, H, W, h, w, gt is not None, info) as pw:
        pw.write("obs", 0, obs_t.numpy())
        pw.write("psf", 0, psf_a)
        if gt is not None:
            pw.write("gt", 0, gt)
        pw.write("alpha", 0, alpha)
    return path


def pack_dataset(data_path, out_path, psf_folder="psf/", obs_folder="obs/", gt_folder="gt/", with_gt=True):
    """Convert a reference-layout dataset folder (all ``n_total`` galaxies, train then test) into one
    GDPACK01 file; returns the path.  Items are read exactly as ``Galaxy_Dataset`` reads them."""
    ds = Galaxy_Dataset(data_path, True, psf_folder, obs_folder, gt_folder)
    if not ds.info:
        raise ValueError(f"no readable info.json under {data_path}")
    n = ds.n_total
    (o0, p0, _), _ = ds.load_item(0)
    H, W, h, w = o0.shape[-2], o0.shape[-1], p0.shape[-2], p0.shape[-1]
    alphas = np.zeros(n, np.float32)
    with PackWriter(out_path, n, H, W, h, w, with_gt, ds.info) as pw:
        for i in range(n):
            (obs, psf, alpha), gt = ds.load_item(i)
            pw.write("obs", i, obs)
            pw.write("psf", i, psf)
            if with_gt:
                pw.write("gt", i, gt)
            alphas[i] = float(alpha.reshape(()))
        pw.write("alpha", 0, alphas)
    return out_path


# ------------------------------------------------------------------ native reader
class PackedGalaxies:
    """A GDPACK01 file opened through the native reader (``gd_pack_*``)."""

    def __init__(self, path, threads=8):
        self.lib = _lib.load()
        self.path = path
        self.threads = int(threads)
        h = ctypes.c_void_p()
        n = ctypes.c_longlong()
        dims = (ctypes.c_int * 5)()
        _lib.check(self.lib.gd_pack_open(path.encode(), ctypes.byref(h), ctypes.byref(n), dims), "gd_pack_open")
        self._h = h
        self.n = n.value
        self.H, self.W, self.h, self.w, self.has_gt = list(dims)
        nb = self.lib.gd_pack_section_bytes(self._h, SECTIONS["info"])
        buf = ctypes.create_string_buffer(max(1, nb))
        _lib.check(self.lib.gd_pack_read(self._h, SECTIONS["info"], 0, 0, buf, 1), "gd_pack_read(info)")
        self.info = json.loads(buf.raw[:nb].decode() or "{}")
        self.n_train = int(self.info.get("n_train", self.n))
        self.n_test = int(self.info.get("n_test", self.n - self.n_train))

    def item_shape(self, section):
        return {"obs": (1, self.H, self.W), "gt": (1, self.H, self.W), "psf": (1, self.h, self.w),
                "alpha": (1, 1, 1)}[section]

    def empty(self, section, count, pin=False):
        return torch.empty((count,) + self.item_shape(section), dtype=torch.float32, pin_memory=pin)

    def read(self, section, g0, count, out=None):
        """Galaxies [g0, g0+count) of a section as a CPU tensor [count, *item] (into ``out`` if given)."""
        out = self.empty(section, count) if out is None else out
        if out.numel() < count * int(np.prod(self.item_shape(section))) or not out.is_contiguous():
            raise ValueError("out too small or not contiguous")
        _lib.check(self.lib.gd_pack_read(self._h, SECTIONS[section], g0, count, out.data_ptr(), self.threads),
                   f"gd_pack_read({section})")
        return out[:count] if out.shape[0] != count else out

    def gather(self, section, idx, out=None):
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.int64))
        out = self.empty(section, len(idx)) if out is None else out
        _lib.check(self.lib.gd_pack_gather(self._h, SECTIONS[section], idx.ctypes.data, len(idx), out.data_ptr(),
                                           self.threads), f"gd_pack_gather({section})")
        return out[:len(idx)]

    def item(self, i):
        """``Galaxy_Dataset.load_item(i)`` from the packed file: ((obs, psf, alpha), gt)."""
        obs, psf, alpha = (self.read(s, i, 1)[0] for s in ("obs", "psf", "alpha"))
        gt = self.read("gt", i, 1)[0] if self.has_gt else None
        return (obs, psf, alpha), gt

    def dataset(self, train=True):
        return PackedGalaxyDataset(self, train)

    def close(self):
        if self._h:
            self.lib.gd_pack_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PackedGalaxyDataset(Dataset):
    """Map-style drop-in for ``Galaxy_Dataset`` over a packed file (same items, same split)."""

    def __init__(self, pack, train=True):
        self.pack, self.train = pack, train

    def __len__(self):
        return self.pack.n_train if self.train else self.pack.n_test

    def __getitem__(self, i):
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self.pack.item(i if self.train else i + self.pack.n_train)


class DeviceBatches:
    """Iterate device batches ``(obs, psf, alpha)`` (+ ``gt`` if ``with_gt``) of a packed file.

    ``indices``: galaxy order (default: ``range(start, stop)``); contiguous runs are read with one
    ranged read per section, anything else with a gather.  ``depth`` pinned host slots are filled
    ahead by a reader thread.  The yielded tensors are fresh device tensors, valid on torch's current
    stream (the H2D copy ran on a side stream the current stream waits on)."""

    def __init__(self, pack, batch_size, device="cuda", start=0, stop=None, indices=None, with_gt=False, depth=2):
        self.pack, self.B = pack, int(batch_size)
        self.device = torch.device(device)
        stop = pack.n if stop is None else stop
        self.idx = np.arange(start, stop, dtype=np.int64) if indices is None else np.asarray(indices, np.int64)
        self.secs = ["obs", "psf", "alpha"] + (["gt"] if with_gt else [])
        if with_gt and not pack.has_gt:
            raise ValueError("packed file has no ground truth")
        self.depth = max(1, int(depth))
        self.stats = {"read_s": 0.0, "bytes": 0}

    def __len__(self):
        return (len(self.idx) + self.B - 1) // self.B

    def _fill(self, slot, b):
        import time
        t0 = time.perf_counter()
        ids = self.idx[b * self.B:(b + 1) * self.B]
        contiguous = len(ids) > 0 and ids[-1] - ids[0] == len(ids) - 1 and np.all(np.diff(ids) == 1)
        for s in self.secs:
            if contiguous:
                self.pack.read(s, int(ids[0]), len(ids), out=slot[s])
            else:
                self.pack.gather(s, ids, out=slot[s])
            self.stats["bytes"] += len(ids) * slot[s][0].numel() * 4
        self.stats["read_s"] += time.perf_counter() - t0
        return len(ids)

    def __iter__(self):
        nb = len(self)
        if nb == 0:
            return
        slots = [{s: self.pack.empty(s, self.B, pin=True) for s in self.secs} for _ in range(self.depth)]
        done_ev = [None] * self.depth          # copy-finished event per slot (slot reusable after it)
        free = queue.Queue()
        ready = queue.Queue()
        for k in range(self.depth):
            free.put(k)
        err = []

        def reader():
            try:
                for b in range(nb):
                    k = free.get()
                    if k is None:
                        return
                    if done_ev[k] is not None:
                        done_ev[k].synchronize()  # the slot's previous H2D copy has landed
                    ready.put((k, self._fill(slots[k], b)))
            except Exception as e:  # surfaced in the consumer
                err.append(e)
                ready.put((None, 0))

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        copy_stream = torch.cuda.Stream(device=self.device)
        cur = torch.cuda.current_stream(self.device)
        try:
            for _ in range(nb):
                k, n = ready.get()
                if k is None:
                    raise err[0]
                out = {}
                with torch.cuda.stream(copy_stream):
                    for s in self.secs:
                        d = torch.empty((n,) + self.pack.item_shape(s), dtype=torch.float32, device=self.device)
                        d.copy_(slots[k][s][:n], non_blocking=True)
                        out[s] = d
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                done_ev[k] = ev
                cur.wait_event(ev)
                for d in out.values():
                    d.record_stream(cur)
                free.put(k)
                batch = (out["obs"], out["psf"], out["alpha"])
                yield (batch, out["gt"]) if "gt" in out else batch
        finally:
            free.put(None)
            th.join(timeout=60)


__all__ = ["Galaxy_Dataset", "get_dataloader", "reference_alpha", "PackWriter", "write_pack", "pack_dataset",
           "PackedGalaxies", "PackedGalaxyDataset", "DeviceBatches", "SECTIONS"]

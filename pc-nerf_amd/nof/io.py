"""On-disk formats either side of the render path, without open3d / python-pcl.

* Point clouds: PCD v0.7 (``DATA ascii`` / ``binary``, float fields; x, y, z selected) -- what the reference
  reads and writes with ``o3d.io.read_point_cloud`` / ``write_point_cloud`` (ipb2dmapping.py:567-590,
  eval_kitti_render.py:1158-1170, print_metrics.py:69-88); KITTI ``velodyne/*.bin`` (x, y, z, intensity float32).
* Ray caches: the 15-column ``self_rays_{train,val}.npy`` + ``self_ranges_*.npy`` (ipb2dmapping.py:455-474,
  828-847) and the two-step ``all_rays_child.npy`` / ``other_interest_sub_nerf_number_child.npy`` /
  ``all_ranges_child.npy`` / ``true_in_all_child.npy`` (eval_kitti_render.py:525-530).  Loaded with
  ``np.load(allow_pickle=False)``.
* Checkpoints: Lightning ``{'state_dict': {'nof_coarse.<key>': ..., 'nof_fine.<key>': ...}}`` or bare state
  dicts (nof_utils.py:176-199 ``extract_model_state_dict`` / ``load_ckpt``), read with
  ``torch.load(weights_only=True)`` -- tensors only, nothing in the file is executed.
"""
from __future__ import annotations

import argparse
import collections
import os
import pickle

import numpy as np
import torch

_PCD_TYPES = {("F", 4): np.float32, ("F", 8): np.float64, ("I", 1): np.int8, ("I", 2): np.int16,
              ("I", 4): np.int32, ("I", 8): np.int64, ("U", 1): np.uint8, ("U", 2): np.uint16,
              ("U", 4): np.uint32, ("U", 8): np.uint64}


def _pcd_header(fh):
    hdr = {}
    while True:
        line = fh.readline()
        if not line:
            raise ValueError("PCD: header ended before DATA")
        s = line.decode("ascii", errors="replace").strip()
        if not s or s.startswith("#"):
            continue
        key, _, val = s.partition(" ")
        hdr[key.upper()] = val.split()
        if key.upper() == "DATA":
            return hdr


def read_pcd(path: str) -> np.ndarray:
    """(N, 3) float32 x, y, z of a PCD file (ascii or binary; binary_compressed is refused)."""
    with open(path, "rb") as fh:
        hdr = _pcd_header(fh)
        fields = hdr["FIELDS"]
        sizes = [int(v) for v in hdr["SIZE"]]
        types = hdr["TYPE"]
        counts = [int(v) for v in hdr.get("COUNT", ["1"] * len(fields))]
        n = int(hdr["POINTS"][0]) if "POINTS" in hdr else int(hdr["WIDTH"][0]) * int(hdr.get("HEIGHT", ["1"])[0])
        kind = hdr["DATA"][0].lower()
        for c in ("x", "y", "z"):
            if c not in fields:
                raise ValueError(f"PCD {path}: no '{c}' field")
        if kind == "binary":
            dt = np.dtype([(f if cnt == 1 else f, _PCD_TYPES[(t, sz)], () if cnt == 1 else (cnt,))
                           for f, t, sz, cnt in zip(fields, types, sizes, counts)])
            buf = fh.read(dt.itemsize * n)
            if len(buf) < dt.itemsize * n:
                raise ValueError(f"PCD {path}: truncated binary data")
            rec = np.frombuffer(buf, dtype=dt, count=n)
            pts = np.stack([rec["x"], rec["y"], rec["z"]], 1)
        elif kind == "ascii":
            cols = np.loadtxt(fh, dtype=np.float64, ndmin=2)
            offs = np.cumsum([0] + counts)
            pts = np.stack([cols[:, offs[fields.index(c)]] for c in ("x", "y", "z")], 1)
        else:
            raise NotImplementedError(f"PCD {path}: DATA {kind} is not supported (ascii and binary are)")
    return np.ascontiguousarray(pts, dtype=np.float32)


def write_pcd(path: str, pts) -> None:
    """Binary xyz float32 PCD with open3d's header layout."""
    p = np.ascontiguousarray(np.asarray(pts, dtype=np.float32).reshape(-1, 3))
    n = p.shape[0]
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z\nSIZE 4 4 4\nTYPE F F F\n"
            f"COUNT 1 1 1\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA binary\n")
    with open(path, "wb") as fh:
        fh.write(head.encode("ascii"))
        fh.write(p.tobytes())


def read_kitti_bin(path: str) -> np.ndarray:
    """KITTI velodyne scan: (N, 4) float32 x, y, z, reflectance."""
    return np.fromfile(path, dtype=np.float32).reshape(-1, 4)


def _load_npy(path):
    return np.load(path, allow_pickle=False)


def load_rays(prefix_dir: str, split: str = "train"):
    """(rays (N, 15) float32, ranges (N, 1) float32) from ``self_rays_<split>.npy`` / ``self_ranges_<split>.npy``."""
    rays = _load_npy(os.path.join(prefix_dir, f"self_rays_{split}.npy")).astype(np.float32, copy=False)
    if rays.ndim != 2 or rays.shape[1] != 15:
        raise ValueError(f"self_rays_{split}.npy must be (N, 15); got {rays.shape}")
    rng_path = os.path.join(prefix_dir, f"self_ranges_{split}.npy")
    ranges = _load_npy(rng_path).astype(np.float32, copy=False).reshape(-1, 1) if os.path.exists(rng_path) \
        else rays[:, 14:15].copy()
    return rays, ranges


def save_rays(prefix_dir: str, rays, ranges=None, split: str = "train") -> None:
    os.makedirs(prefix_dir, exist_ok=True)
    rays = np.asarray(rays, dtype=np.float32)
    np.save(os.path.join(prefix_dir, f"self_rays_{split}.npy"), rays)
    np.save(os.path.join(prefix_dir, f"self_ranges_{split}.npy"),
            np.asarray(rays[:, 14:15] if ranges is None else ranges, dtype=np.float32).reshape(-1, 1))


def load_view_rows(dir_: str):
    """Two-step inputs of one test frame: rows (M, 13) float32, other (M,) int64, ranges (M,) float32,
    true_in (M,) bool (any of the latter three may be None when absent)."""
    rows = _load_npy(os.path.join(dir_, "all_rays_child.npy")).astype(np.float32, copy=False)
    if rows.ndim != 2 or rows.shape[1] != 13:
        raise ValueError(f"all_rays_child.npy must be (M, 13); got {rows.shape}")

    def opt(name, dtype):
        p = os.path.join(dir_, name)
        return _load_npy(p).reshape(-1).astype(dtype) if os.path.exists(p) else None

    return (rows, opt("other_interest_sub_nerf_number_child.npy", np.int64), opt("all_ranges_child.npy", np.float32),
            opt("true_in_all_child.npy", bool))


def save_view_rows(dir_: str, rows, other, ranges=None, true_in=None) -> None:
    os.makedirs(dir_, exist_ok=True)
    np.save(os.path.join(dir_, "all_rays_child.npy"), np.asarray(rows, dtype=np.float32))
    np.save(os.path.join(dir_, "other_interest_sub_nerf_number_child.npy"),
            np.asarray(other, dtype=np.int64).reshape(-1, 1))
    if ranges is not None:
        np.save(os.path.join(dir_, "all_ranges_child.npy"), np.asarray(ranges, dtype=np.float32).reshape(-1, 1))
    if true_in is not None:
        np.save(os.path.join(dir_, "true_in_all_child.npy"), np.asarray(true_in, dtype=np.float32).reshape(-1, 1))


# Non-tensor globals a Lightning checkpoint of the reference can hold besides what torch allows by default:
# save_hyperparameters(argparse.Namespace) (train_kitti.py:23) and Lightning's AttributeDict (a dict subclass)
# under its module paths across Lightning versions -- rebuilt as a plain OrderedDict, nothing of Lightning
# imported or executed.  Each is a data container whose reconstruction runs no code of the file.
_CKPT_SAFE_GLOBALS = [argparse.Namespace] + [(collections.OrderedDict, n) for n in (
    "pytorch_lightning.utilities.parsing.AttributeDict", "lightning_fabric.utilities.data.AttributeDict",
    "lightning.fabric.utilities.data.AttributeDict", "lightning.pytorch.utilities.parsing.AttributeDict")]


def load_checkpoint(ckpt_path: str) -> dict:
    """torch.load(weights_only=True) -- the file never executes anything -- retried with the data-container
    globals above allowed when the checkpoint carries them (a full Lightning checkpoint: hyper_parameters,
    optimizer / lr-scheduler states, callbacks, loops)."""
    try:
        return torch.load(ckpt_path, map_location="cpu", weights_only=True)
    except pickle.UnpicklingError:
        with torch.serialization.safe_globals(_CKPT_SAFE_GLOBALS):
            return torch.load(ckpt_path, map_location="cpu", weights_only=True)


def extract_model_state_dict(ckpt_path: str, model_name: str = "model", prefixes_to_ignore=()):
    """nof_utils.py:176-191: the ``model_name.``-prefixed entries of a (Lightning) checkpoint, prefix removed."""
    ck = load_checkpoint(ckpt_path)
    if "state_dict" in ck:
        ck = ck["state_dict"]
    out = {}
    for k, v in ck.items():
        if not k.startswith(model_name):
            continue
        k = k[len(model_name) + 1:]
        if any(k.startswith(p) for p in prefixes_to_ignore):
            continue
        out[k] = v
    return out


def load_ckpt(model, ckpt_path: str, model_name: str = "model", prefixes_to_ignore=()) -> None:
    """nof_utils.py:194-199."""
    sd = model.state_dict()
    sd.update(extract_model_state_dict(ckpt_path, model_name, prefixes_to_ignore))
    model.load_state_dict(sd)


def save_ckpt(path: str, **models) -> None:
    """Lightning-layout checkpoint: ``save_ckpt(p, nof_coarse=m1, nof_fine=m2)``."""
    sd = {}
    for name, m in models.items():
        for k, v in m.state_dict().items():
            sd[f"{name}.{k}"] = v.detach().cpu()
    torch.save({"state_dict": sd}, path)

"""``tensorflow_datasets``-compatible loaders (tf_dist_example.py:15,27-29).

There is no network on the training hosts, so ``load('mnist')`` returns a deterministic SYNTHETIC
MNIST-shaped dataset (60,000 train / 10,000 test, uint8 [28,28,1] images, int64 labels) unless
real MNIST IDX files are found in ``$TDL_DATA_DIR``, ``~/tensorflow_datasets/mnist`` or
``~/.keras/datasets`` (``train-images-idx3-ubyte[.gz]`` etc.).  The synthetic images are class
prototypes (random stroke blobs per digit) plus noise and random shifts, so models actually
learn on them (loss decreases, accuracy rises above chance).
"""
from __future__ import annotations

import gzip
import os
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .dataset import Dataset

_PROGRESS = [True]


def disable_progress_bar():
    _PROGRESS[0] = False


def enable_progress_bar():
    _PROGRESS[0] = True


@dataclass
class SplitInfo:
    name: str
    num_examples: int


@dataclass
class DatasetInfo:
    name: str
    splits: Dict[str, SplitInfo] = field(default_factory=dict)
    features: Dict[str, object] = field(default_factory=dict)
    supervised_keys: Tuple[str, str] = ("image", "label")
    synthetic: bool = True
    description: str = ""

    @property
    def num_classes(self):
        return 10


def _find_idx(name: str) -> Optional[str]:
    dirs = [os.environ.get("TDL_DATA_DIR", ""), os.path.expanduser("~/tensorflow_datasets/mnist"),
            os.path.expanduser("~/.keras/datasets"), os.path.expanduser("~/.keras/datasets/mnist")]
    for d in dirs:
        if not d:
            continue
        for suf in ("", ".gz"):
            p = os.path.join(d, name + suf)
            if os.path.exists(p):
                return p
    return None


def _read_idx(path: str) -> np.ndarray:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[:4], "big")
    nd = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(nd)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


def synthetic_mnist(n: int, seed: int = 0, num_classes: int = 10):
    """Deterministic learnable MNIST-shaped data: uint8 [n,28,28], int64 labels [n]."""
    rng = np.random.default_rng(12345)  # prototypes are fixed across splits
    yy, xx = np.mgrid[0:28, 0:28]
    protos = np.zeros((num_classes, 28, 28), np.float32)
    for c in range(num_classes):
        for _ in range(4):  # 4 gaussian strokes per class
            cy, cx = rng.uniform(7, 21, 2)
            sy, sx = rng.uniform(1.5, 4.5, 2)
            protos[c] += np.exp(-(((yy - cy) / sy) ** 2 + ((xx - cx) / sx) ** 2))
        protos[c] /= protos[c].max()
    r = np.random.default_rng(seed)
    labels = r.integers(0, num_classes, n)
    imgs = protos[labels]
    shifts = r.integers(-2, 3, (n, 2))
    out = np.empty((n, 28, 28), np.float32)
    for s0 in range(-2, 3):
        for s1 in range(-2, 3):
            m = (shifts[:, 0] == s0) & (shifts[:, 1] == s1)
            if m.any():
                out[m] = np.roll(np.roll(imgs[m], s0, axis=1), s1, axis=2)
    out = out * r.uniform(0.7, 1.0, (n, 1, 1)) + r.normal(0, 0.15, out.shape)
    return (np.clip(out, 0, 1) * 255).astype(np.uint8), labels.astype(np.int64)


def mnist_arrays(split: str = "train"):
    """(images uint8 [n,28,28], labels int64 [n]) — real IDX files if present, else synthetic."""
    stem = "train" if split.startswith("train") else "t10k"
    pi, pl = _find_idx(f"{stem}-images-idx3-ubyte"), _find_idx(f"{stem}-labels-idx1-ubyte")
    if pi and pl:
        return _read_idx(pi), _read_idx(pl).astype(np.int64), False
    n = 60000 if stem == "train" else 10000
    x, y = synthetic_mnist(n, seed=0 if stem == "train" else 1)
    return x, y, True


def load(name: str, split=None, as_supervised: bool = False, with_info: bool = False, data_dir=None,
         download: bool = True, shuffle_files: bool = False, batch_size=None, **kw):
    name = name.split(":")[0].lower()
    if name not in ("mnist", "fashion_mnist"):
        raise ValueError(f"dataset {name!r} is not available offline (supported: mnist)")
    splits = {}
    info = DatasetInfo(name)
    for sp in ("train", "test"):
        x, y, synth = mnist_arrays(sp)
        x = torch.from_numpy(x.reshape(-1, 28, 28, 1).copy())
        yt = torch.from_numpy(y)
        ds = Dataset.from_tensor_slices((x, yt) if as_supervised else {"image": x, "label": yt})
        if batch_size:
            ds = ds.batch(batch_size)
        splits[sp] = ds
        info.splits[sp] = SplitInfo(sp, len(x))
        info.synthetic = synth
    info.features = {"image": ("uint8", (28, 28, 1)), "label": ("int64", ())}
    if split is not None:
        out = [splits[s] for s in split] if isinstance(split, (list, tuple)) else splits[split]
    else:
        out = splits
    return (out, info) if with_info else out

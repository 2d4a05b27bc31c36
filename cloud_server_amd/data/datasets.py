"""Datasets: user-uploaded JPEG folders + tag.json, MNIST idx files, synthetic MNIST.

Reference loaders:
* ``read_user_data`` (construct_distribute.py:424-463) — tag.json maps ``<basename>.jpg``
  to a digit; images are found by walking the (hard-coded) ``data`` dir; ordered
  train/test split at ``int(N*ratio)`` with no shuffle before the split.
* ``input_data.read_data_sets`` (construct_distribute_url.py:355) — stock MNIST idx.gz.
* ``DataSet`` (construct_distribute.py:466-569) — flatten to 784, scale to [0,1],
  epoch-shuffled ``next_batch`` with wrap-around.

Here a dataset is decoded ONCE into a uint8 ``[N, 784]`` array plus int64 labels.  On the
MI355X it is uploaded once and stays resident in HBM (MNIST is 47 MB even as fp32; the
288 GB HBM3E makes residency free); batches are gathered on device by index
(``BatchStream``), so the training loop never touches the host.
"""
from __future__ import annotations

import gzip
import json
import os
import struct
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

IMAGE_EXTS = (".jpg", ".jpeg", ".png", ".bmp")


@dataclass
class ArrayDataset:
    images: np.ndarray   # uint8 [N, 784]
    labels: np.ndarray   # int64 [N]

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    def split(self, ratio: float) -> Tuple["ArrayDataset", "ArrayDataset"]:
        """Ordered split at int(N*ratio) (construct_distribute.py:455-460)."""
        mid = int(len(self) * ratio)
        return (ArrayDataset(self.images[:mid], self.labels[:mid]),
                ArrayDataset(self.images[mid:], self.labels[mid:]))


def decode_image(path: str, size: int = 28) -> np.ndarray:
    """Grayscale decode -> uint8 [size*size]. Non-28x28 inputs are resized (bicubic)."""
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("L")
        if im.size != (size, size):
            im = im.resize((size, size), Image.BICUBIC)
        return np.asarray(im, dtype=np.uint8).reshape(-1)


def walk_images(root: str) -> List[str]:
    out = []
    for dirpath, dirs, files in os.walk(root):
        dirs.sort()
        for f in sorted(files):
            if f.lower().endswith(IMAGE_EXTS):
                out.append(os.path.join(dirpath, f))
    return out


def load_user_data(data_dir: str, tag_path: str) -> ArrayDataset:
    """All labelled images under ``data_dir`` (labels keyed by basename, as in tag.json)."""
    with open(tag_path, "r", encoding="utf-8") as f:
        tags: Dict[str, str] = json.load(f)
    imgs, labels = [], []
    for p in walk_images(data_dir):
        key = os.path.basename(p)
        if key not in tags:
            rel = os.path.relpath(p, data_dir)
            if rel not in tags:
                continue
            key = rel
        try:
            lab = int(tags[key])
        except (TypeError, ValueError):
            continue
        if not 0 <= lab <= 9:
            continue
        imgs.append(decode_image(p))
        labels.append(lab)
    if not imgs:
        return ArrayDataset(np.zeros((0, 784), np.uint8), np.zeros((0,), np.int64))
    return ArrayDataset(np.stack(imgs), np.asarray(labels, dtype=np.int64))


def _open_maybe_gz(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    """IDX file (MNIST format): magic 0x0000 08 <ndim>, big-endian dims, uint8 payload."""
    with _open_maybe_gz(path) as f:
        magic = struct.unpack(">I", f.read(4))[0]
        if (magic >> 8) != 0x08:
            raise ValueError(f"{path}: not a uint8 IDX file (magic {magic:#x})")
        ndim = magic & 0xFF
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        data = np.frombuffer(f.read(), dtype=np.uint8).copy()   # writable (torch.from_numpy)
    return data.reshape(dims)


def _find(d: str, stem: str) -> Optional[str]:
    for name in (stem, stem + ".gz"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    for dirpath, _, files in os.walk(d):
        for f in files:
            if f.startswith(stem):
                return os.path.join(dirpath, f)
    return None


def load_mnist_dir(d: str) -> Tuple[ArrayDataset, Optional[ArrayDataset]]:
    """Stock MNIST (the URL datatype, test-data/test-url.txt): train + optional test split."""
    ti, tl = _find(d, "train-images-idx3-ubyte"), _find(d, "train-labels-idx1-ubyte")
    if ti is None or tl is None:
        raise FileNotFoundError(f"no MNIST train idx files under {d}")
    train = ArrayDataset(read_idx(ti).reshape(-1, 784), read_idx(tl).astype(np.int64))
    vi, vl = _find(d, "t10k-images-idx3-ubyte"), _find(d, "t10k-labels-idx1-ubyte")
    test = None
    if vi and vl:
        test = ArrayDataset(read_idx(vi).reshape(-1, 784), read_idx(vl).astype(np.int64))
    return train, test


def write_idx(path: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    hdr = struct.pack(">I", 0x0800 | arr.ndim) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(hdr + arr.tobytes())


def synthetic_mnist(n: int, seed: int = 0) -> ArrayDataset:
    """MNIST-shaped synthetic data (random strokes over noise) with learnable labels:
    the class sets a spatial template so a model can fit it (used by bench and tests)."""
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, 10, size=n).astype(np.int64)
    yy, xx = np.mgrid[0:28, 0:28]
    templates = np.zeros((10, 28, 28), np.float32)
    for c in range(10):
        cy, cx = 6 + (c // 5) * 14 + 2, 3 + (c % 5) * 5 + 2
        templates[c] = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 10.0)
    noise = rng.random((n, 28, 28), dtype=np.float32) * 0.35
    imgs = np.clip(templates[labels] * 0.9 + noise, 0, 1)
    return ArrayDataset((imgs * 255).astype(np.uint8).reshape(n, 784), labels)


def load_dataset_for_model(data_dir: str, tag_path: Optional[str], datatype: str) -> ArrayDataset:
    """``datatype`` = 'url' (MNIST idx under data_dir) or 'file' (JPEGs + tag.json)."""
    if datatype == "url":
        train, test = load_mnist_dir(data_dir)
        if test is not None:
            return ArrayDataset(np.concatenate([train.images, test.images]),
                                np.concatenate([train.labels, test.labels]))
        return train
    if tag_path is None:
        raise FileNotFoundError("file datatype needs a tag.json")
    return load_user_data(data_dir, tag_path)

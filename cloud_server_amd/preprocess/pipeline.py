"""Preprocessing pipeline over a model workspace (reference PreprocessView.execute).

Reference flow (apps/preprocess/views.py:49-137): copy the dataset into
``model/<m>/data``, then for each operation in order and for each image listed in
``tag.json``: resize to 28x28 (in place), apply the op either in place
(``overlap`` false) or into a ``<name>_copy<ext>`` twin whose label is appended to
tag.json (``overlap`` true).  Every op re-reads and re-writes JPEG files.

Here the listed images are decoded ONCE into a ``uint8 [N, 28, 28]`` batch, every op runs
on the whole batch (batched HIP kernels on the MI355X, ``preprocess.gpu``; NumPy
reference otherwise), and the results are encoded once at the end.  Semantics kept:
ops see the copies created by earlier ops (the tag map is re-read per op in the
reference); a repeated ``_copy`` name is overwritten; ``overlap`` is honoured for JSON
``true`` and the string ``"true"`` (reference quirk 9 compared with ``is``).
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import ops_ref

JPEG_QUALITY = 95   # cv2.imwrite default


def copied_name(name: str) -> str:
    """preprocess.py:8-15."""
    root, ext = os.path.splitext(name)
    return root + "_copy" + ext


def _read(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("L"), dtype=np.uint8)


def _write(path: str, arr: np.ndarray) -> None:
    from PIL import Image
    im = Image.fromarray(np.ascontiguousarray(arr, dtype=np.uint8), mode="L")
    ext = os.path.splitext(path)[1].lower()
    if ext in (".jpg", ".jpeg"):
        im.save(path, quality=JPEG_QUALITY)
    else:
        im.save(path)


def copy_dataset(src: str, dst: str) -> None:
    """``cp -R <data>/* <model>/data`` (views.py:73-75) without a shell."""
    os.makedirs(dst, exist_ok=True)
    if os.path.isfile(src):
        shutil.copy2(src, dst)
        return
    for name in os.listdir(src):
        s, d = os.path.join(src, name), os.path.join(dst, name)
        if os.path.isdir(s):
            shutil.copytree(s, d, dirs_exist_ok=True)
        else:
            shutil.copy2(s, d)


def is_overlap(op: Dict[str, Any]) -> bool:
    v = op.get("overlap")
    return v is True or v == "true"


def _backend_apply(backend: str):
    if backend in ("gpu", "auto"):
        try:
            from . import gpu
            if gpu.available():
                return gpu.apply_op
        except Exception:
            if backend == "gpu":
                raise
    return ops_ref.apply_op


def run(data_dir: str, tag_path: str, operations: Sequence[Dict[str, Any]], backend: str = "auto",
        mode: str = "saturate", seed: Optional[int] = None, size: int = 28) -> Dict[str, str]:
    """Apply ``operations`` to the images listed in ``tag_path`` (paths relative to
    ``data_dir``).  Returns the updated tag map (also written to ``tag_path``)."""
    with open(tag_path, "r", encoding="utf-8") as f:
        tags: Dict[str, str] = json.load(f)
    for op in operations:
        name = op.get("operationName", "")
        if ops_ref.OP_MAP.get(name, name) not in ops_ref.OP_NAMES:
            raise ValueError(f"unknown operation {name!r}")
    apply = _backend_apply(backend)
    rng = np.random.default_rng(seed)
    images: Dict[str, np.ndarray] = {}
    dirty = set()

    def load(rel: str) -> np.ndarray:
        if rel not in images:
            p = os.path.join(data_dir, rel)
            if not os.path.exists(p):
                raise FileNotFoundError(rel)
            a = _read(p)
            if a.shape != (size, size):
                a = ops_ref.resize(a, size)[0]      # views.py:121 resizes before each op
                dirty.add(rel)
            images[rel] = a
        return images[rel]

    for op in operations:
        names = [n for n in tags if os.path.exists(os.path.join(data_dir, n)) or n in images]
        if not names:
            continue
        batch = np.stack([load(n) for n in names])
        out = apply(ops_ref.OP_MAP.get(op["operationName"], op["operationName"]), batch,
                    op.get("value1"), op.get("value2"), mode=mode, rng=rng)
        overlap = is_overlap(op)
        new_tags = dict(tags)
        for i, n in enumerate(names):
            tgt = copied_name(n) if overlap else n
            images[tgt] = out[i]
            dirty.add(tgt)
            if overlap:
                new_tags[tgt] = tags[n]
        tags = new_tags
    for rel in dirty:
        p = os.path.join(data_dir, rel)
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        _write(p, images[rel])
    with open(tag_path, "w", encoding="utf-8") as f:
        json.dump(tags, f, ensure_ascii=False)
    return tags

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
import torch

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


def _backend(backend: str):
    """'gpu' (required), 'cpu', or 'auto' (GPU kernels when a device is present)."""
    if backend in ("gpu", "auto"):
        from . import gpu
        if gpu.available():
            return gpu
        if backend == "gpu":
            raise RuntimeError("preprocess backend 'gpu' requested but no HIP device/kernels")
    return None


def run(data_dir: str, tag_path: str, operations: Sequence[Dict[str, Any]], backend: str = "auto",
        mode: str = "saturate", seed: Optional[int] = None, size: int = 28) -> Dict[str, str]:
    """Apply ``operations`` to the images listed in ``tag_path`` (paths relative to
    ``data_dir``).  Returns the updated tag map (also written to ``tag_path``).

    The image set is one uint8 [N, size, size] batch (device-resident on the GPU
    backend): decoded once, every op is one batched call over the rows of the names
    currently in the tag map, results are encoded once at the end."""
    with open(tag_path, "r", encoding="utf-8") as f:
        tags: Dict[str, str] = json.load(f)
    for op in operations:
        name = op.get("operationName", "")
        if ops_ref.OP_MAP.get(name, name) not in ops_ref.OP_NAMES:
            raise ValueError(f"unknown operation {name!r}")
    dev = _backend(backend)
    rng = np.random.default_rng(seed)
    row: Dict[str, int] = {}          # name -> row of ``batch``
    dirty = set()

    # decode every listed image that exists (resize to size x size, views.py:121)
    names = [n for n in tags if os.path.exists(os.path.join(data_dir, n))]
    imgs = []
    for n in names:
        a = _read(os.path.join(data_dir, n))
        if a.shape != (size, size):
            a = (dev.resize(a[None], size) if dev is not None else ops_ref.resize(a, size))[0]
            dirty.add(n)
        row[n] = len(imgs)
        imgs.append(a)
    batch = np.stack(imgs) if imgs else np.zeros((0, size, size), np.uint8)
    if dev is not None:
        batch = dev.to_device(batch)
    apply = dev.apply_op if dev is not None else ops_ref.apply_op

    def take(rows):
        return batch[torch.as_tensor(rows, device=batch.device)] if dev is not None else batch[rows]

    def cat(parts):
        return torch.cat(parts) if dev is not None else np.concatenate(parts)

    for op in operations:
        cur = [n for n in tags if n in row]
        if not cur:
            continue
        fname = ops_ref.OP_MAP.get(op["operationName"], op["operationName"])

        def call(x):
            return apply(fname, x, op.get("value1"), op.get("value2"), mode=mode, rng=rng)

        if not is_overlap(op):
            idx = [row[n] for n in cur]
            out = call(take(idx))
            if dev is not None:
                batch[torch.as_tensor(idx, device=batch.device)] = out
            else:
                batch[idx] = out
            dirty.update(cur)
            continue
        # overlap: the reference walks the tag map in order, so an image whose ``_copy``
        # twin was (re)written earlier in this same op reads that fresh twin.  Resolve
        # those chains level by level; each level is one batched call.
        pos = {n: i for i, n in enumerate(cur)}
        src = {}
        for n in cur:
            base, ext = os.path.splitext(n)
            if base.endswith("_copy"):
                m = base[:-5] + ext
                if m in pos and pos[m] < pos[n]:
                    src[n] = m
        level = {}
        for n in cur:
            level[n] = level[src[n]] + 1 if n in src else 0
        outs: Dict[str, Any] = {}
        for L in range(max(level.values()) + 1):
            names_l = [n for n in cur if level[n] == L]
            if L == 0:
                x = take([row[n] for n in names_l])
            else:
                x = cat([outs[src[n]][None] for n in names_l])
            y = call(x)
            for i, n in enumerate(names_l):
                outs[n] = y[i]
        new_tags = dict(tags)
        fresh, fresh_rows = [], []
        for n in cur:
            tgt = copied_name(n)
            new_tags[tgt] = tags[n]
            dirty.add(tgt)
            if tgt in row:                          # a repeated _copy name is overwritten
                batch[row[tgt]] = outs[n]
            else:
                row[tgt] = len(row)
                fresh.append(outs[n][None])
        if fresh:
            batch = cat([batch] + fresh)
        tags = new_tags
    host = batch.cpu().numpy() if dev is not None else batch
    for rel in dirty:
        p = os.path.join(data_dir, rel)
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        _write(p, host[row[rel]])
    with open(tag_path, "w", encoding="utf-8") as f:
        json.dump(tags, f, ensure_ascii=False)
    return tags

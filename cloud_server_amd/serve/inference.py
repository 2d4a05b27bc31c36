"""Digit inference with a warm per-model cache.

Reference (C25/C28): every request copied ``construct_inference.py`` to the cluster host
over SFTP, started a fresh ``python3`` + TF process that rebuilt the graph, restored the
max-step checkpoint and ran one argmax on ``/cpu:0``, then downloaded ``result.json``
into a single global path shared by all users (apps/construction/views.py:198-268,
construct_inference.py:293-347).

Here a model is loaded once per (owner, model, checkpoint step) and kept on the device
(MI355X when present) in an LRU cache; each request is a single forward pass.

Image preparation is the reference's (construct_inference.py:312-330): grayscale,
resize to 20x20, centred in a 28x28 canvas (offset 4), pixels > 150 -> 254 else 0 (the
100 < v <= 150 branch writes into a discarded array, so the result is a binarisation),
divide by 255.  ``prep="mnist"`` instead feeds the plain 28x28 grayscale image /255 —
the distribution the model was trained on.
"""
from __future__ import annotations

import io
import json
import os
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.cnn import DigitNet
from ..models.dsl import parse_train_config
from ..runtime import checkpoint as ckpt

FAIL_NO_MODEL = {"result": "fail", "message": "no model please train a model first"}


def prepare_reference(img_bytes: bytes) -> np.ndarray:
    """-> float32 [784] exactly as construct_inference.py:312-330."""
    from PIL import Image
    with Image.open(io.BytesIO(img_bytes)) as im:
        im = im.convert("L").resize((20, 20), Image.BICUBIC)
        arr = np.asarray(im, dtype=np.float32)
    canvas = np.zeros((28, 28), np.float32)
    canvas[4:24, 4:24] = np.where(arr > 150, 254.0, 0.0)
    return (canvas / 255.0).reshape(-1)


def prepare_mnist(img_bytes: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(img_bytes)) as im:
        im = im.convert("L")
        if im.size != (28, 28):
            im = im.resize((28, 28), Image.BICUBIC)
        return (np.asarray(im, dtype=np.float32) / 255.0).reshape(-1)


class InferenceService:
    def __init__(self, device: Optional[str] = None, capacity: int = 32):
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.capacity = capacity
        self._cache: "OrderedDict[Tuple[str, int], DigitNet]" = OrderedDict()
        self._lock = threading.Lock()
        self.hits = self.misses = 0

    def _load(self, model_dir: str) -> Optional[DigitNet]:
        last = ckpt.latest(model_dir)
        if last is None:
            return None
        step, path = last
        key = (os.path.abspath(model_dir), step)
        with self._lock:
            net = self._cache.get(key)
            if net is not None:
                self._cache.move_to_end(key)
                self.hits += 1
                return net
        obj = ckpt.load(path)
        cfg = parse_train_config(json.loads(obj["config"]))
        net = DigitNet(cfg.plan(), device=self.device, bn_mode=cfg.bn_mode)
        net.import_state(obj["model"])
        net.eval()
        with self._lock:
            self.misses += 1
            # drop older checkpoints of the same model
            for k in [k for k in self._cache if k[0] == key[0]]:
                del self._cache[k]
            self._cache[key] = net
            while len(self._cache) > self.capacity:
                self._cache.popitem(last=False)
        return net

    @torch.no_grad()
    def predict_arrays(self, model_dir: str, x: np.ndarray) -> Optional[np.ndarray]:
        net = self._load(model_dir)
        if net is None:
            return None
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(self.device)
        return net(t.view(-1, 784)).argmax(1).cpu().numpy()

    def predict(self, model_dir: str, img_bytes: bytes, prep: str = "reference") -> Dict[str, str]:
        fn = prepare_reference if prep == "reference" else prepare_mnist
        try:
            x = fn(img_bytes)
        except Exception as exc:
            return {"result": "fail", "message": f"cannot decode image: {exc}"}
        out = self.predict_arrays(model_dir, x[None])
        if out is None:
            return dict(FAIL_NO_MODEL)
        return {"result": "success", "message": str(int(out[0]))}

    async def predict_async(self, model_dir: str, img_bytes: bytes, prep: str = "reference") -> Dict[str, str]:
        """``predict`` off the event loop (decode + forward run in the threadpool)."""
        from starlette.concurrency import run_in_threadpool
        return await run_in_threadpool(self.predict, model_dir, img_bytes, prep)

    def predict_many(self, model_dir: str, images: Sequence[bytes], prep: str = "reference") -> List[Dict[str, str]]:
        fn = prepare_reference if prep == "reference" else prepare_mnist
        xs = np.stack([fn(b) for b in images]) if images else np.zeros((0, 784), np.float32)
        out = self.predict_arrays(model_dir, xs)
        if out is None:
            return [dict(FAIL_NO_MODEL) for _ in images]
        return [{"result": "success", "message": str(int(v))} for v in out]

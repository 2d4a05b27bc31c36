"""Digit inference with a warm per-model cache.

Reference (C25/C28): every request copied ``construct_inference.py`` to the cluster host
over SFTP, started a fresh ``python3`` + TF process that rebuilt the graph, restored the
max-step checkpoint and ran one argmax on ``/cpu:0``, then downloaded ``result.json``
into a single global path shared by all users (apps/construction/views.py:198-268,
construct_inference.py:293-347).

Here a model is loaded once per (owner, model, checkpoint step) and kept on the device
(MI355X when present) in an LRU cache.  On the GPU the forward is the HIP training
forward captured per batch bucket (``serve.hip_infer``), and concurrent requests for one
model are MICRO-BATCHED: a per-(model, prep) batcher thread drains every request that
arrived while the previous batch ran and serves them with one graph replay.  Server-side
latencies are kept (``latency_ms``) for the serving benchmark.

Image preparation is the reference's (construct_inference.py:312-330): grayscale,
resize to 20x20, centred in a 28x28 canvas (offset 4), pixels > 150 -> 254 else 0 (the
100 < v <= 150 branch writes into a discarded array, so the result is a binarisation),
divide by 255.  ``prep="mnist"`` instead feeds the plain 28x28 grayscale image /255 —
the distribution the model was trained on.
"""
from __future__ import annotations

import asyncio
import io
import json
import os
import queue
import threading
import time
import weakref
from collections import OrderedDict, deque
from concurrent.futures import Future
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

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


def decode_reference_u8(img_bytes: bytes) -> np.ndarray:
    """The host half of the reference prep: grayscale + bicubic 20x20 -> uint8 [400]
    (centring + binarisation run on the device, ``csa_img_infer_prep_u8``)."""
    from PIL import Image
    with Image.open(io.BytesIO(img_bytes)) as im:
        return np.asarray(im.convert("L").resize((20, 20), Image.BICUBIC), dtype=np.uint8).reshape(-1)


def decode_mnist_u8(img_bytes: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(img_bytes)) as im:
        im = im.convert("L")
        if im.size != (28, 28):
            im = im.resize((28, 28), Image.BICUBIC)
        return np.asarray(im, dtype=np.uint8).reshape(-1)


class BatcherClosed(RuntimeError):
    """The batcher's model entry was replaced (newer checkpoint / LRU eviction)."""


class _Batcher:
    """Micro-batching: one thread per (model, prep) takes the first queued request, then
    every request already waiting (up to ``max_batch``) and runs them as ONE batch.

    ``close`` and ``submit`` serialise on a lock: every request enqueued before the close
    sentinel is still served, and a ``submit`` after ``close`` raises ``BatcherClosed``
    (the caller re-resolves the model entry) instead of parking a Future behind the
    sentinel of an exited thread."""

    def __init__(self, fn: Callable[[np.ndarray], np.ndarray], max_batch: int = 256):
        self.fn, self.max_batch = fn, max_batch
        self.q: "queue.Queue[Optional[Tuple[np.ndarray, Future]]]" = queue.Queue()
        self.batches = self.items = 0
        self.closed = False
        self._lk = threading.Lock()
        self.t = threading.Thread(target=self._loop, name="csa-infer-batch", daemon=True)
        self.t.start()

    def submit(self, x: np.ndarray) -> Future:
        f: Future = Future()
        with self._lk:
            if self.closed:
                raise BatcherClosed("model entry replaced")
            self.q.put((x, f))
        return f

    def close(self) -> None:
        with self._lk:
            if self.closed:
                return
            self.closed = True
            self.q.put(None)

    def _serve(self, items) -> None:
        try:
            out = self.fn(np.stack([x for x, _ in items]))
            for (_, f), v in zip(items, out):
                f.set_result(int(v))
        except Exception as exc:            # every waiter sees the failure
            for _, f in items:
                if not f.done():
                    f.set_exception(exc)
        self.batches += 1
        self.items += len(items)

    def _loop(self) -> None:
        while True:
            first = self.q.get()
            if first is None:
                return
            items = [first]
            stop = False
            while len(items) < self.max_batch:
                try:
                    it = self.q.get_nowait()
                except queue.Empty:
                    break
                if it is None:
                    stop = True
                    break
                items.append(it)
            self._serve(items)
            if stop:
                return


def prepare_mnist(img_bytes: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(img_bytes)) as im:
        im = im.convert("L")
        if im.size != (28, 28):
            im = im.resize((28, 28), Image.BICUBIC)
        return (np.asarray(im, dtype=np.float32) / 255.0).reshape(-1)


class _Entry:
    def __init__(self, net: DigitNet, cfg, hip):
        self.net, self.cfg, self.hip = net, cfg, hip
        self.batchers: Dict[str, _Batcher] = {}
        self.retired = False

    def retire(self) -> None:
        """Dropped from the cache (caller holds the service lock): close its batchers and
        drop them — each batcher's callback holds this entry, so the dict closed a
        reference cycle that only a gen-2 collection would have freed."""
        self.retired = True
        for bt in self.batchers.values():
            bt.close()
        self.batchers = {}


_LIVE: "weakref.WeakSet[InferenceService]" = weakref.WeakSet()


def close_all() -> None:
    """Retire every live service's cached models (their HIP graphs and batcher threads) in
    the calling thread — e.g. before a process goes on to capture graphs of its own."""
    for svc in list(_LIVE):
        svc.close()


class InferenceService:
    def __init__(self, device: Optional[str] = None, capacity: int = 32, use_hip: bool = True):
        _LIVE.add(self)
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", 0)
        self.capacity = capacity
        self.use_hip = use_hip
        self._cache: "OrderedDict[Tuple[str, int], _Entry]" = OrderedDict()
        self._lock = threading.Lock()
        self._loading: Dict[str, threading.Lock] = {}
        self.hits = self.misses = 0
        self.lat = deque(maxlen=20000)      # server-side seconds per request (decode -> digit)
        self.hip_error = ""

    def _lookup(self, key) -> Optional[_Entry]:
        with self._lock:
            ent = self._cache.get(key)
            if ent is not None:
                self._cache.move_to_end(key)
                self.hits += 1
            return ent

    def _entry(self, model_dir: str) -> Optional[_Entry]:
        last = ckpt.latest(model_dir)
        if last is None:
            return None
        step, path = last
        key = (os.path.abspath(model_dir), step)
        ent = self._lookup(key)
        if ent is not None:
            return ent
        with self._lock:
            load_lock = self._loading.setdefault(key[0], threading.Lock())
        with load_lock:                      # one load (and one set of captures) per model
            ent = self._lookup(key)
            if ent is not None:
                return ent
            ent = self._load_entry(path)
            with self._lock:
                if self._loading.get(key[0]) is load_lock:
                    del self._loading[key[0]]        # (waiters hold their own reference)
                self.misses += 1
                # drop older checkpoints of the same model
                for k in [k for k in self._cache if k[0] == key[0]]:
                    self._cache.pop(k).retire()
                self._cache[key] = ent
                while len(self._cache) > self.capacity:
                    _, old = self._cache.popitem(last=False)
                    old.retire()
        return ent

    def _load_entry(self, path: str) -> _Entry:
        obj = ckpt.load(path)
        cfg = parse_train_config(json.loads(obj["config"]))
        hip = None
        if self.use_hip and self.device.type == "cuda":
            from .hip_infer import try_build
            try:
                hip = try_build(cfg, obj["model"], self.device)
            except Exception as exc:        # outside the HIP family: eager torch forward
                self.hip_error = repr(exc)
                hip = None
        if hip is not None:
            net = hip.state.model           # ONE resident copy of the weights per entry
        else:
            net = DigitNet(cfg.plan(), device=self.device, bn_mode=cfg.bn_mode)
            net.import_state(obj["model"])
            net.eval()
        return _Entry(net, cfg, hip)

    def _load(self, model_dir: str) -> Optional[DigitNet]:
        ent = self._entry(model_dir)
        return ent.net if ent is not None else None

    def backend(self, model_dir: str) -> str:
        ent = self._entry(model_dir)
        return "none" if ent is None else ("hip" if ent.hip is not None else f"torch:{self.device.type}")

    # ---- batched forward of uint8 inputs (the serving path) ----
    def _run_u8(self, ent: _Entry, x: np.ndarray, prep: str) -> np.ndarray:
        if ent.hip is not None:
            return ent.hip.predict_u8(x, prep)
        if prep == "reference":                 # host completion of the reference prep
            canvas = np.zeros((x.shape[0], 28, 28), np.float32)
            canvas[:, 4:24, 4:24] = np.where(x.reshape(-1, 20, 20) > 150, 254.0, 0.0)
            xf = canvas.reshape(-1, 784) / 255.0
        else:
            xf = x.astype(np.float32) / 255.0
        with torch.no_grad():
            t = torch.from_numpy(np.ascontiguousarray(xf, dtype=np.float32)).to(self.device)
            return ent.net(t.view(-1, 784)).argmax(1).cpu().numpy()

    def _batcher(self, ent: _Entry, prep: str) -> _Batcher:
        with self._lock:
            if ent.retired:
                raise BatcherClosed("model entry replaced")
            b = ent.batchers.get(prep)
            if b is None:
                b = ent.batchers[prep] = _Batcher(lambda xs, e=ent, p=prep: self._run_u8(e, xs, p))
            return b

    def _submit(self, model_dir: str, x: np.ndarray, prep: str) -> Optional[Future]:
        """Queue one decoded image on the current entry's batcher.  An entry replaced
        between lookup and submit (a newer checkpoint loaded by another request) closed
        its batchers: look the model up again and queue on the new entry."""
        for _ in range(8):
            ent = self._entry(model_dir)
            if ent is None:
                return None
            try:
                return self._batcher(ent, prep).submit(x)
            except BatcherClosed:
                continue
        raise RuntimeError("model entry kept changing while submitting")

    @staticmethod
    def _decode(img_bytes: bytes, prep: str) -> np.ndarray:
        return decode_reference_u8(img_bytes) if prep == "reference" else decode_mnist_u8(img_bytes)

    @torch.no_grad()
    def predict_arrays(self, model_dir: str, x: np.ndarray) -> Optional[np.ndarray]:
        """Float inputs [n, 784] in [0, 1].  Exact u8/255 images take the HIP path."""
        ent = self._entry(model_dir)
        if ent is None:
            return None
        x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 784)
        u8 = np.rint(x * 255.0)
        if ent.hip is not None and np.array_equal(u8 / 255.0, x.astype(np.float64)) and u8.min() >= 0 and u8.max() <= 255:
            return ent.hip.predict_u8(u8.astype(np.uint8), "mnist")
        t = torch.from_numpy(x).to(self.device)
        return ent.net(t).argmax(1).cpu().numpy()

    def predict(self, model_dir: str, img_bytes: bytes, prep: str = "reference") -> Dict[str, str]:
        t0 = time.perf_counter()
        prep = "reference" if prep == "reference" else "mnist"
        try:
            x = self._decode(img_bytes, prep)
        except Exception as exc:
            return {"result": "fail", "message": f"cannot decode image: {exc}"}
        fut = self._submit(model_dir, x, prep)
        if fut is None:
            return dict(FAIL_NO_MODEL)
        v = fut.result()
        self.lat.append(time.perf_counter() - t0)
        return {"result": "success", "message": str(int(v))}

    async def predict_async(self, model_dir: str, img_bytes: bytes, prep: str = "reference") -> Dict[str, str]:
        """Decode in the threadpool, then await the model's micro-batcher (the event loop
        never blocks on the device)."""
        from starlette.concurrency import run_in_threadpool
        t0 = time.perf_counter()
        prep = "reference" if prep == "reference" else "mnist"
        try:
            x = await run_in_threadpool(self._decode, img_bytes, prep)
        except Exception as exc:
            return {"result": "fail", "message": f"cannot decode image: {exc}"}
        fut = await run_in_threadpool(self._submit, model_dir, x, prep)
        if fut is None:
            return dict(FAIL_NO_MODEL)
        v = await asyncio.wrap_future(fut)
        self.lat.append(time.perf_counter() - t0)
        return {"result": "success", "message": str(int(v))}

    def predict_many(self, model_dir: str, images: Sequence[bytes], prep: str = "reference") -> List[Dict[str, str]]:
        prep = "reference" if prep == "reference" else "mnist"
        ent = self._entry(model_dir)
        if ent is None:
            return [dict(FAIL_NO_MODEL) for _ in images]
        if not images:
            return []
        out = self._run_u8(ent, np.stack([self._decode(b, prep) for b in images]), prep)
        return [{"result": "success", "message": str(int(v))} for v in out]

    def latency_ms(self) -> Dict[str, Any]:
        v = sorted(self.lat)
        if not v:
            return {"n": 0}
        q = lambda p: 1e3 * v[min(len(v) - 1, int(p * len(v)))]
        return {"n": len(v), "p50": q(0.5), "p90": q(0.9), "p99": q(0.99)}

    def close(self) -> None:
        with self._lock:
            for ent in self._cache.values():
                ent.retire()
            self._cache.clear()

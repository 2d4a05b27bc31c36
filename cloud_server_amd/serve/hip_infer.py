"""GPU inference through the hand-written HIP forward kernels, captured per batch bucket.

Reference path (C25/C28, apps/construction/views.py:198-268 -> construct_inference.py:
293-347): a fresh TF process per request, one image, argmax on ``/cpu:0``.

Here a model's forward is the TRAINING program's forward (``HipProgram._forward``: the
fused conv pair, BN-apply + activation folded into the consumers, MFMA dense layers) with
BatchNorm on its running statistics, plus a logits GEMM and an argmax, captured ONCE per
batch bucket into a HIP graph.  A request batch is:

    pinned host staging -> H2D (one copy) -> graph replay -> D2H of the [n] argmax

The reference's image prep (resize 20x20 on the host decoder, then centre in 28x28 and
binarise at 150 -> 254) runs on the device inside the graph (``csa_img_infer_prep_u8``)
and writes the uint8 canvas the forward kernels read like a dataset row (u8 / 255 is the
reference's float input exactly).  ``prep="mnist"`` uploads the 28x28 uint8 image itself.
"""
from __future__ import annotations

import dataclasses
import threading
from typing import Dict, List, Optional

import numpy as np
import torch

from ..data.datasets import ArrayDataset
from ..models.dsl import TrainConfig

BUCKETS = (1, 4, 16, 64, 256)


def bucket_for(n: int) -> int:
    for b in BUCKETS:
        if n <= b:
            return b
    return BUCKETS[-1]


class _Bucket:
    """One captured forward of ``B`` rows for one prep kind."""

    def __init__(self, cfg: TrainConfig, state: Dict[str, torch.Tensor], B: int, device: torch.device,
                 prep: str):
        from ..runtime.engine import TrainEngine
        from ..runtime.hip_program import HipProgram
        from ..ops import fused as K
        self.B, self.prep, self.device = B, prep, device
        dummy = ArrayDataset(np.zeros((B, 784), np.uint8), np.zeros(B, np.int64))
        c = dataclasses.replace(cfg, batch_size=B)
        self.eng = eng = TrainEngine(c, dummy, device=device, backend="hip", use_graph=False)
        if not isinstance(eng.program, HipProgram):
            raise RuntimeError(f"no HIP lowering: {eng.fallback_reason}")
        eng.model.import_state(state)
        eng.model.eval()
        eng.stream.rows[0].copy_(torch.arange(B, device=device))    # row r reads input r
        eng.stream.cursor.zero_()
        self.logits = torch.zeros(B, 10, device=device)
        self.pred = torch.zeros(B, dtype=torch.int64, device=device)
        # host staging (pinned) and its device twin
        shape = (B, 400) if prep == "reference" else (B, 784)
        self.h_in = torch.zeros(shape, dtype=torch.uint8, pin_memory=True)
        self.d_in = torch.zeros(shape, dtype=torch.uint8, device=device)
        self.h_out = torch.zeros(B, dtype=torch.int64, pin_memory=True)
        self._lib = K
        from ..preprocess import gpu as G
        self._G = G
        self.graph = None
        self._capture()

    def _body(self) -> None:
        img = self.eng.data.images
        if self.prep == "reference":
            rc = self._G._lib().csa_img_infer_prep_u8(self.d_in.data_ptr(), img.data_ptr(), self.B,
                                                      self._lib.stream())
            if rc != 0:
                raise RuntimeError(f"csa_img_infer_prep_u8 failed: {rc}")
        else:
            img.copy_(self.d_in)
        self.eng.program.predict_logits_into(self.logits)
        torch.argmax(self.logits, dim=1, out=self.pred)

    def _capture(self) -> None:
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._body()                      # warm-up (library init, allocator)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g

    def run(self, x: np.ndarray) -> np.ndarray:
        """``x`` uint8 [n, 400] (reference: 20x20 decoded) or [n, 784] (mnist), n <= B."""
        n = x.shape[0]
        self.h_in[:n].numpy()[...] = x
        if n < self.B:
            self.h_in[n:].zero_()
        self.d_in.copy_(self.h_in, non_blocking=True)
        self.graph.replay()
        self.h_out.copy_(self.pred, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return self.h_out[:n].numpy().copy()


class HipPredictor:
    """All buckets of one (model, checkpoint): built lazily, one lock (one stream)."""

    def __init__(self, cfg: TrainConfig, state: Dict[str, torch.Tensor], device: torch.device):
        self.cfg, self.state, self.device = cfg, state, device
        self._buckets: Dict[tuple, _Bucket] = {}
        self.lock = threading.Lock()

    def predict_u8(self, x: np.ndarray, prep: str) -> np.ndarray:
        out: List[np.ndarray] = []
        with self.lock, torch.cuda.device(self.device):
            i = 0
            while i < x.shape[0]:
                n = min(x.shape[0] - i, BUCKETS[-1])
                B = bucket_for(n)
                key = (B, prep)
                b = self._buckets.get(key)
                if b is None:
                    b = self._buckets[key] = _Bucket(self.cfg, self.state, B, self.device, prep)
                out.append(b.run(x[i:i + n]))
                i += n
        return np.concatenate(out) if out else np.zeros(0, np.int64)


def try_build(cfg: TrainConfig, state: Dict[str, torch.Tensor], device: torch.device) -> Optional[HipPredictor]:
    """A HIP predictor when the device is a GPU and the net lowers to the HIP kernels."""
    if device.type != "cuda":
        return None
    p = HipPredictor(cfg, state, device)
    p.predict_u8(np.zeros((1, 400), np.uint8), "reference")      # raises if it cannot lower
    return p

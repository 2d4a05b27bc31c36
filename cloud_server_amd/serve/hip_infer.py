"""GPU inference through the hand-written HIP forward kernels, captured per batch bucket.

Reference path (C25/C28, apps/construction/views.py:198-268 -> construct_inference.py:
293-347): a fresh TF process per request, one image, argmax on ``/cpu:0``.

Here a model is loaded ONCE per (model, checkpoint) into a resident weight state — one
``DigitNet`` holding the flat parameters and the BatchNorm running statistics on the
serving GPU — and every batch bucket runs the training program's forward
(``HipProgram(forward_only=True)``: the fused conv pair, BN-apply + activation folded
into the consumers, MFMA dense layers) over THOSE weights, plus a logits GEMM and an
argmax.  A bucket owns only its activations and its I/O staging; there is no gradient,
optimizer or batch-stream state anywhere on the serving path.

Every bucket of both preps is captured into a HIP graph when the model loads, in
``thread_local`` capture mode and under a process-wide capture lock — never lazily on a
request thread — so concurrent GPU work from other threads of the API process (another
model's batcher, GPU preprocessing) can neither invalidate a capture nor be broken by
one.  A request batch is:

    pinned host staging -> H2D (one copy) -> graph replay -> D2H of the [n] argmax

The reference's image prep (resize 20x20 on the host decoder, then centre in 28x28 and
binarise at 150 -> 254) runs on the device inside the graph (``csa_img_infer_prep_u8``)
and writes the uint8 canvas the forward kernels read like a dataset row (u8 / 255 is the
reference's float input exactly).  ``prep="mnist"`` uploads the 28x28 uint8 image itself.
"""
from __future__ import annotations

import dataclasses
import threading
from types import SimpleNamespace
from typing import Dict, List, Optional

import numpy as np
import torch

from ..models.dsl import TrainConfig
from ..utils.graphs import capture

BUCKETS = (1, 4, 16, 64, 256)
PREPS = ("reference", "mnist")

# Graph captures AND graph destructions in this process are serialised: thread_local
# capture mode keeps other threads' unrelated GPU calls legal during a capture, but a
# graph executable destroyed while a capture is in progress aborts the process (see
# utils/graphs.py), and a retired model's buckets may die on any request thread.
CAPTURE_LOCK = threading.RLock()


def bucket_for(n: int) -> int:
    for b in BUCKETS:
        if n <= b:
            return b
    return BUCKETS[-1]


class ServeState:
    """A model's resident forward state on one device: flat weights + BN running stats."""

    def __init__(self, cfg: TrainConfig, state: Dict[str, torch.Tensor], device: torch.device):
        from ..models.cnn import DigitNet
        self.cfg, self.device = cfg, device
        self.model = DigitNet(cfg.plan(), device=device, seed=cfg.seed, bn_mode=cfg.bn_mode)
        self.model.import_state(state)
        self.model.eval()
        self.flat = self.model.flat.data


class _FwdEngine:
    """The engine surface ``HipProgram(forward_only=True)`` reads: config, device, the
    shared model/weights, a disabled distributed context, and a dataset/stream of ``B``
    rows that are simply the bucket's input buffer (row r reads input r)."""

    def __init__(self, st: ServeState, B: int):
        from ..parallel.dist import DistContext
        dev = st.device
        self.cfg = dataclasses.replace(st.cfg, batch_size=B)
        self.device, self.model, self.flat = dev, st.model, st.flat
        self.flat_grad = None
        self.ctx = DistContext(device=dev)
        self.data = SimpleNamespace(images=torch.zeros(B, 784, dtype=torch.uint8, device=dev),
                                    labels=torch.zeros(B, dtype=torch.int64, device=dev))
        self.stream = SimpleNamespace(rows=torch.arange(B, device=dev).view(1, B),
                                      cursor=torch.zeros(1, dtype=torch.int64, device=dev), wrap=1)


class _Bucket:
    """One captured forward of ``B`` rows for one prep kind over a shared ServeState."""

    def __init__(self, st: ServeState, B: int, prep: str):
        from ..runtime.hip_program import HipProgram
        from ..ops import fused as K
        from ..preprocess import gpu as G
        self.B, self.prep, self.device = B, prep, st.device
        self.eng = _FwdEngine(st, B)
        self.program = HipProgram(self.eng, forward_only=True)
        dev = st.device
        self.logits = torch.zeros(B, 10, device=dev)
        self.pred = torch.zeros(B, dtype=torch.int64, device=dev)
        shape = (B, 400) if prep == "reference" else (B, 784)
        self.h_in = torch.zeros(shape, dtype=torch.uint8, pin_memory=True)   # host staging
        self.d_in = torch.zeros(shape, dtype=torch.uint8, device=dev)
        self.h_out = torch.zeros(B, dtype=torch.int64, pin_memory=True)
        self._K, self._G = K, G
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._capture()

    def _body(self) -> None:
        img = self.eng.data.images
        if self.prep == "reference":
            rc = self._G._lib().csa_img_infer_prep_u8(self.d_in.data_ptr(), img.data_ptr(), self.B,
                                                      self._K.stream())
            if rc != 0:
                raise RuntimeError(f"csa_img_infer_prep_u8 failed: {rc}")
        else:
            img.copy_(self.d_in)
        self.program.predict_logits_into(self.logits)
        torch.argmax(self.logits, dim=1, out=self.pred)

    def _capture(self) -> None:
        with CAPTURE_LOCK:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._body()                      # warm-up (library init, lazy buffers)
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with capture(g):
                self._body()
            self.graph = g

    def __del__(self):
        g, self.graph = getattr(self, "graph", None), None
        if g is not None:
            with CAPTURE_LOCK:          # never destroyed while another thread captures
                del g

    def logits_u8(self, x: np.ndarray) -> torch.Tensor:
        """Replay on ``x`` (n <= B rows) and return the [n, 10] logits (device tensor, a
        view of this bucket's output: copy before the next replay)."""
        n = x.shape[0]
        self.h_in[:n].numpy()[...] = x
        if n < self.B:
            self.h_in[n:].zero_()
        self.d_in.copy_(self.h_in, non_blocking=True)
        self.graph.replay()
        return self.logits[:n]

    def run(self, x: np.ndarray) -> np.ndarray:
        """``x`` uint8 [n, 400] (reference: 20x20 decoded) or [n, 784] (mnist), n <= B."""
        n = x.shape[0]
        self.logits_u8(x)
        self.h_out.copy_(self.pred, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return self.h_out[:n].numpy().copy()


class HipPredictor:
    """Every bucket of one (model, checkpoint), captured at construction; one lock."""

    def __init__(self, cfg: TrainConfig, state: Dict[str, torch.Tensor], device: torch.device,
                 buckets=BUCKETS, preps=PREPS):
        self.cfg, self.device = cfg, device
        self.lock = threading.Lock()
        with torch.cuda.device(device):
            self.state = ServeState(cfg, state, device)
            self._buckets: Dict[tuple, _Bucket] = {(B, p): _Bucket(self.state, B, p)
                                                   for B in buckets for p in preps}
        self.buckets = tuple(buckets)

    def _bucket(self, n: int, prep: str) -> _Bucket:
        for B in self.buckets:
            if n <= B:
                return self._buckets[(B, prep)]
        return self._buckets[(self.buckets[-1], prep)]

    def predict_u8(self, x: np.ndarray, prep: str) -> np.ndarray:
        out: List[np.ndarray] = []
        with self.lock, torch.cuda.device(self.device):
            i, cap = 0, self.buckets[-1]
            while i < x.shape[0]:
                n = min(x.shape[0] - i, cap)
                out.append(self._bucket(n, prep).run(x[i:i + n]))
                i += n
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def logits_u8(self, x: np.ndarray, prep: str) -> np.ndarray:
        """[n, 10] fp32 logits of ``x`` (n <= the largest bucket): the numerics check."""
        with self.lock, torch.cuda.device(self.device):
            return self._bucket(x.shape[0], prep).logits_u8(x).cpu().numpy()


def try_build(cfg: TrainConfig, state: Dict[str, torch.Tensor], device: torch.device) -> Optional[HipPredictor]:
    """A HIP predictor when the device is a GPU and the net lowers to the HIP kernels
    (raises ``Unsupported`` otherwise; the caller falls back to the eager forward)."""
    if device.type != "cuda":
        return None
    return HipPredictor(cfg, state, device)

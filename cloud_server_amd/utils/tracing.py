"""Tracing and step timing (the reference only timed ``sess.run`` with
``time.time()`` around it, construct_distribute.py:412-414).

* ``trace_range(name)`` — a ROCTx range (``librocprofiler-sdk-roctx``), visible in
  ``rocprofv3 --marker-trace`` timelines next to the kernels; a no-op unless
  ``CSA_TRACE=1`` (ranges around graph replays cost a few hundred ns each).
* ``mark(msg)`` — a ROCTx instant marker.
* ``PhaseTimer`` — HIP-event timing of named phases on the current stream, read back
  lazily (no host sync in the timed region), exported into the metrics JSONL.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, List, Optional, Tuple

_ROCTX = None
_TRIED = False


def _roctx():
    global _ROCTX, _TRIED
    if _TRIED:
        return _ROCTX
    _TRIED = True
    if os.environ.get("CSA_TRACE", "0") != "1":
        return None
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        for d in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(d + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                return lib
            except OSError:
                continue
    return None


def enabled() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(msg: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


class PhaseTimer:
    """Per-phase device time via HIP events (CUDA-API names in torch)."""

    def __init__(self, device=None, enabled: bool = True):
        import torch
        self.enabled = enabled and torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
        self._pending: List[Tuple[str, object, object]] = []
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            with trace_range(name):
                yield
            self._add(name, (time.perf_counter() - t0) * 1e3)
            return
        import torch
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        with trace_range(name):
            yield
        b.record()
        self._pending.append((name, a, b))

    def _add(self, name: str, ms: float) -> None:
        self.totals[name] = self.totals.get(name, 0.0) + ms
        self.counts[name] = self.counts.get(name, 0) + 1

    def collect(self) -> Dict[str, float]:
        """Mean ms per phase since the last collect (syncs on the recorded events)."""
        for name, a, b in self._pending:
            b.synchronize()
            self._add(name, a.elapsed_time(b))
        self._pending.clear()
        out = {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}
        self.totals.clear()
        self.counts.clear()
        return out

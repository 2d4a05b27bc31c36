"""HIP-graph capture that no Python finalizer can interrupt.

Root cause of the round-2 GPU-suite abort (profiles/r3_gpu_suite_abort.md): objects
from an earlier engine — its ``CUDAGraph``s, in reference cycles with the engine — were
finalised by the cyclic garbage collector at whatever allocation happened to trigger a
collection, which was sometimes INSIDE a later capture (the DP tuner's timing graphs).
Destroying a graph executable while this thread is capturing aborts the process in the
HIP runtime (SIGABRT, rc 134), with only an unrelated Python frame on the stack.
PyTorch's ``torch.cuda.graph`` no longer collects before capturing by default, so every
capture in this package goes through ``capture()``: collect first, keep the collector
off until the capture has ended, and always use ``thread_local`` capture mode so the
RCCL watchdog's event queries and other threads' GPU calls stay legal meanwhile.
"""
from __future__ import annotations

import contextlib
import gc
from typing import Iterator, Optional

import torch


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", stream: Optional["torch.cuda.Stream"] = None,
            pool=None) -> Iterator[None]:
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        kw = {} if stream is None else {"stream": stream}
        if pool is not None:
            kw["pool"] = pool
        with torch.cuda.graph(graph, capture_error_mode="thread_local", **kw):
            yield
    finally:
        if was:
            gc.enable()

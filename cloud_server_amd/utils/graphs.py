"""HIP-graph capture that no Python finalizer can interrupt.

Root cause of the round-2 GPU-suite abort (profiles/r3_gpu_suite_abort.md): objects
from an earlier engine — its ``CUDAGraph``s, in reference cycles with the engine — were
finalised by the cyclic garbage collector at whatever allocation happened to trigger a
collection, which was sometimes INSIDE a later capture (the DP tuner's timing graphs).
Destroying a graph executable while this thread is capturing aborts the process in the
HIP runtime (SIGABRT, rc 134), with only an unrelated Python frame on the stack.
So every capture in this package goes through ``capture()``: the collector is off until
the capture has ended (a pending cycle is collected later, outside any capture), and the
capture always uses ``thread_local`` mode so the RCCL watchdog's event queries and other
threads' GPU calls stay legal meanwhile.

(An explicit ``gc.collect()`` before every capture was the first fix; it made each
re-capture of the packed host cost ~40 ms of collection — 83-100 ms per admission /
retirement instead of 7-10 ms, profiles/r3_multitenant.md — and is not needed for the
invariant: with the collector disabled nothing finalises cyclic garbage mid-capture.)
"""
from __future__ import annotations

import contextlib
import gc
import threading
from typing import Iterator, Optional

import torch

# the collector's enable flag is process state: captures on different threads overlap, so
# it is switched off by the first capture to start and back on by the LAST one to end
_lock = threading.Lock()
_active = 0
_was_enabled = False


def _enter() -> None:
    global _active, _was_enabled
    with _lock:
        if _active == 0:
            _was_enabled = gc.isenabled()
            gc.disable()
        _active += 1


def _exit() -> None:
    global _active
    with _lock:
        _active -= 1
        if _active == 0 and _was_enabled:
            gc.enable()


def active_captures() -> int:
    return _active


# RCCL watchdog (round 4): the process-group watchdog thread polls the end events of
# eager collectives until it reaps them, about every 100 ms.  A capture that contains an
# RCCL collective pulls RCCL's internal stream into the capture, and a query of an event
# recorded on a stream that is capturing NOW fails (hipErrorCapturedEvent) and aborts the
# process — seen in the GPU suite whenever a capture began within the watchdog's poll of
# the warm-up's collectives.  So a capture under an initialised RCCL process group first
# drains the device and gives the watchdog time to reap every completed eager work.
_WATCHDOG_DRAIN_S = 0.3


def _drain_rccl_watchdog() -> None:
    import time
    try:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
            return
    except Exception:  # pragma: no cover
        return
    torch.cuda.synchronize()
    time.sleep(_WATCHDOG_DRAIN_S)


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", stream: Optional["torch.cuda.Stream"] = None,
            pool=None) -> Iterator[None]:
    _drain_rccl_watchdog()
    _enter()
    try:
        kw = {} if stream is None else {"stream": stream}
        if pool is not None:
            kw["pool"] = pool
        with torch.cuda.graph(graph, capture_error_mode="thread_local", **kw):
            yield
    finally:
        _exit()

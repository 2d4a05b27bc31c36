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


# (round 4 drained the device and slept 0.3 s here before every capture under RCCL, to let
# the process-group watchdog reap eager collectives first; captured collectives now run on
# a dedicated process group that never carries an eager work the watchdog is polling —
# parallel/dp.py GradSync._setup_capture_group — so capture needs no wait at all)


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", stream: Optional["torch.cuda.Stream"] = None,
            pool=None) -> Iterator[None]:
    _enter()
    try:
        kw = {} if stream is None else {"stream": stream}
        if pool is not None:
            kw["pool"] = pool
        with torch.cuda.graph(graph, capture_error_mode="thread_local", **kw):
            yield
    finally:
        _exit()

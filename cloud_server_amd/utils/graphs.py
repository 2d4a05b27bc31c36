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


def wait_retired(group=None, timeout_s: float = 10.0) -> Optional[bool]:
    """Block until the process-group watchdog has retired every eager collective of
    ``group`` (default: the default group) — none left in the flight recorder's active
    list.  True once retired, False on timeout, None where there is nothing to wait for
    (no RCCL group, or the flight recorder off: TORCH_NCCL_TRACE_BUFFER_SIZE=0)."""
    import json
    import os
    import time
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    try:
        from torch._C._distributed_c10d import _dump_nccl_trace_json
    except ImportError:  # pragma: no cover
        return None
    if int(os.environ.get("TORCH_NCCL_TRACE_BUFFER_SIZE", "0") or 0) <= 0:
        return None
    if os.environ.get("TORCH_NCCL_BLOCKING_WAIT", "0") == "1":
        return None      # no watchdog thread exists (tests/test_gpu_rccl_threads.py), so
                         # nothing queries a captured event
    if group is None:
        if dist.get_backend() != "nccl":
            return None
        group = dist.distributed_c10d._get_default_group()
    name = str(dist.distributed_c10d._get_process_group_name(group))

    def mine(e) -> bool:
        pg = e.get("process_group")
        if isinstance(pg, (list, tuple)) and pg:
            pg = pg[0]
        elif isinstance(pg, dict):
            pg = pg.get("name", pg.get("pg_name"))
        return str(pg) == name
    t0 = time.perf_counter()
    while True:
        try:
            dump = json.loads(_dump_nccl_trace_json(includeCollectives=True, onlyActive=True))
        except Exception:  # pragma: no cover - dump format / availability
            return None
        if not any(mine(e) for e in dump.get("entries", [])):
            return True
        if time.perf_counter() - t0 > timeout_s:
            return False
        time.sleep(0.002)


# Before every capture under RCCL, the default group's eager collectives must be RETIRED by
# its watchdog (an observable condition: the flight recorder's active list, not a timed
# sleep).  Round 5 found why the dedicated capture group alone was not enough: torch hands
# out the capture stream, side streams and every process group's RCCL stream from ONE
# round-robin pool of 32 streams per device, so a capture can run on the very stream an
# eager default-group collective just used — the watchdog's query of that collective's end
# event then aborts the process (hipErrorCapturedEvent; 2 of 10 world-1 DP bench runs,
# scripts/gpu_r5c3.sh).  Captured collectives still go to the capture group
# (parallel/dp.py GradSync._setup_capture_group), so no default-group work is issued
# while capturing.


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", stream: Optional["torch.cuda.Stream"] = None,
            pool=None) -> Iterator[None]:
    if _active == 0:
        wait_retired()
    _enter()
    try:
        if stream is None and torch.cuda.is_available():
            # outside torch's stream pool: never the stream of an RCCL group (utils/streams.py)
            from .streams import capture_stream
            stream = capture_stream()
        kw = {} if stream is None else {"stream": stream}
        if pool is not None:
            kw["pool"] = pool
        with torch.cuda.graph(graph, capture_error_mode="thread_local", **kw):
            yield
    finally:
        _exit()

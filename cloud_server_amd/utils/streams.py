"""Streams that never alias a process group's RCCL stream.

torch hands out ``torch.cuda.Stream()`` objects, ``torch.cuda.graph``'s default capture
stream AND every ProcessGroupNCCL's internal RCCL stream from one round-robin pool of 32
streams per device.  So a capture, or a side stream joined into one, can run on the very
HIP stream that an eager default-group collective just used.  The process-group watchdog
then queries that collective's end event on a capturing stream, and the process aborts
(hipErrorCapturedEvent).  Round 5 saw this in 2 of 6 world-1 bench runs of the overlapped
all-reduce program, whose bucket side stream is part of every capture
(``scripts/gpu_r5c3.sh``).

Every stream that takes part in a capture here is therefore created with
``hipStreamCreateWithFlags`` (non-blocking, outside torch's pool) and wrapped as a
``torch.cuda.ExternalStream``.  Streams are created once and never destroyed (a handful
per process).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict

import torch

_lock = threading.Lock()
_capture: Dict[int, "torch.cuda.ExternalStream"] = {}
_hip = None


def _lib():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        _hip.hipStreamCreateWithFlags.restype = ctypes.c_int
        _hip.hipSetDevice.argtypes = [ctypes.c_int]
        _hip.hipSetDevice.restype = ctypes.c_int
        _hip.hipGetDevice.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _hip.hipGetDevice.restype = ctypes.c_int
    return _hip


def dedicated_stream(device) -> "torch.cuda.ExternalStream":
    """A new non-blocking stream on ``device`` that is not in torch's stream pool."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    torch.cuda.init()
    lib = _lib()
    prev = ctypes.c_int(0)
    lib.hipGetDevice(ctypes.byref(prev))
    try:
        if prev.value != idx:
            lib.hipSetDevice(idx)
        s = ctypes.c_void_p()
        rc = lib.hipStreamCreateWithFlags(ctypes.byref(s), 1)       # hipStreamNonBlocking
        if rc != 0:
            raise RuntimeError(f"hipStreamCreateWithFlags failed ({rc})")
    finally:
        if prev.value != idx:
            lib.hipSetDevice(prev.value)
    return torch.cuda.ExternalStream(s.value, device=torch.device("cuda", idx))


def capture_stream(device=None) -> "torch.cuda.ExternalStream":
    """The process's capture stream for ``device`` (one per device, created on first use)."""
    idx = torch.device(device).index if device is not None else torch.cuda.current_device()
    if idx is None:
        idx = torch.cuda.current_device()
    with _lock:
        s = _capture.get(idx)
        if s is None:
            s = _capture[idx] = dedicated_stream(torch.device("cuda", idx))
        return s

"""GPU-slot scheduler: Python face of ``libcsa_runtime.so`` (csrc/runtime/scheduler.cpp).

Policy (see the C++ header comment): per-GPU slots, least-loaded placement, FIFO with
bounded head-of-line skipping, multi-GPU jobs take distinct GPUs.  ``PyScheduler``
implements the identical policy in Python and is used when the native library is not
built (e.g. a minimal CPU install); tests run both against each other.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from collections import deque
from typing import List, Optional, Tuple

from ..ops import build as _build


class NativeScheduler:
    def __init__(self, ngpu: int, slots_per_gpu: int = 4, max_skip: int = 8):
        path = _build.build_runtime()        # stamp-checked: rebuilds only a stale library
        lib = C.CDLL(path)
        lib.csa_sched_create.restype = C.c_void_p
        lib.csa_sched_create.argtypes = [C.c_int, C.c_int, C.c_int]
        lib.csa_sched_destroy.argtypes = [C.c_void_p]
        lib.csa_sched_submit.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        lib.csa_sched_next.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int), C.c_int]
        lib.csa_sched_release.argtypes = [C.c_void_p, C.c_int64]
        lib.csa_sched_cancel.argtypes = [C.c_void_p, C.c_int64]
        lib.csa_sched_reserve.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        lib.csa_sched_load.argtypes = [C.c_void_p, C.c_int]
        lib.csa_sched_queued.argtypes = [C.c_void_p]
        self.lib = lib
        self.h = lib.csa_sched_create(ngpu, slots_per_gpu, max_skip)
        if not self.h:
            raise ValueError("bad scheduler parameters")
        self.ngpu = ngpu

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.csa_sched_destroy(self.h)
            self.h = None

    def submit(self, job: int, ngpus: int = 1) -> bool:
        return self.lib.csa_sched_submit(self.h, job, ngpus) == 0

    def next(self) -> Optional[Tuple[int, List[int]]]:
        j = C.c_int64()
        buf = (C.c_int * self.ngpu)()
        n = self.lib.csa_sched_next(self.h, C.byref(j), buf, self.ngpu)
        return (int(j.value), list(buf[:n])) if n > 0 else None

    def release(self, job: int) -> int:
        return self.lib.csa_sched_release(self.h, job)

    def cancel(self, job: int) -> bool:
        return bool(self.lib.csa_sched_cancel(self.h, job))

    def reserve(self, job: int, gpu: int) -> bool:
        return self.lib.csa_sched_reserve(self.h, job, gpu) == 0

    def load(self, gpu: int) -> int:
        return self.lib.csa_sched_load(self.h, gpu)

    def queued(self) -> int:
        return self.lib.csa_sched_queued(self.h)


class PyScheduler:
    def __init__(self, ngpu: int, slots_per_gpu: int = 4, max_skip: int = 8):
        if ngpu <= 0 or slots_per_gpu <= 0:
            raise ValueError("bad scheduler parameters")
        self.ngpu, self.slots, self.max_skip = ngpu, slots_per_gpu, max(0, max_skip)
        self._load = [0] * ngpu
        self._owners: List[List[int]] = [[] for _ in range(ngpu)]
        self._q: deque = deque()
        self._mu = threading.Lock()

    def submit(self, job: int, ngpus: int = 1) -> bool:
        if ngpus <= 0 or ngpus > self.ngpu:
            return False
        with self._mu:
            self._q.append([job, ngpus, 0])
        return True

    def _pick(self, n: int) -> List[int]:
        free = [g for g in range(self.ngpu) if self._load[g] < self.slots]
        if len(free) < n:
            return []
        free.sort(key=lambda g: self._load[g])      # stable: ties keep lowest id
        return sorted(free[:n])

    def next(self):
        with self._mu:
            for i, (job, n, _) in enumerate(self._q):
                g = self._pick(n)
                if g:
                    if i > 0 and self._q[0][2] >= self.max_skip:
                        return None
                    for j in range(i):
                        self._q[j][2] += 1
                    for x in g:
                        self._load[x] += 1
                        self._owners[x].append(job)
                    del self._q[i]
                    return job, g
        return None

    def release(self, job: int) -> int:
        with self._mu:
            n = 0
            for g in range(self.ngpu):
                if job in self._owners[g]:
                    self._owners[g].remove(job)
                    self._load[g] -= 1
                    n += 1
            return n

    def cancel(self, job: int) -> bool:
        with self._mu:
            for i, it in enumerate(self._q):
                if it[0] == job:
                    del self._q[i]
                    return True
        return False

    def reserve(self, job: int, gpu: int) -> bool:
        with self._mu:
            if not 0 <= gpu < self.ngpu or self._load[gpu] >= self.slots:
                return False
            self._load[gpu] += 1
            self._owners[gpu].append(job)
            return True

    def load(self, gpu: int) -> int:
        return self._load[gpu] if 0 <= gpu < self.ngpu else -1

    def queued(self) -> int:
        return len(self._q)


def make_scheduler(ngpu: int, slots_per_gpu: int = 4, max_skip: int = 8):
    try:
        return NativeScheduler(ngpu, slots_per_gpu, max_skip)
    except Exception:
        return PyScheduler(ngpu, slots_per_gpu, max_skip)

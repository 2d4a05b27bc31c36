"""Asynchronous, bounded-staleness parameter server ("async_ps") — the reference's own
data-parallel semantics, as an option beside the synchronous strategies of ``dp.py``.

Reference (construct_distribute.py:344-357, 402-414): ``replica_device_setter`` puts every
variable on ``/job:ps``; each worker pulls the variables, runs forward/backward on its
batch and pushes its gradients; the PS applies ``ApplyAdagrad`` to each push as it
arrives.  There is no barrier between workers, so a gradient may have been computed on
parameters that other workers' pushes have since changed (stale gradients).

Here every rank is a worker AND the owner ("PS task") of one contiguous shard of the flat
parameter buffer, with that shard's optimizer slots (as in the sharded ``ps`` strategy).
One step of rank r at clock t:

1. **push**   — its gradient g_r(t) (its own batch mean: each push is one worker's update,
   as on the reference PS; no 1/W averaging) goes, shard by shard, to every owner;
2. **apply**  — as owner it applies arrived pushes ONE BY ONE (an optimizer update each, in
   (clock, source) order) — every push with clock <= t - s must be applied (it waits for
   them), newer ones are applied only if they have already arrived;
3. **publish** — its shard's current parameters, tagged with its *applied-through* clock
   (every push of every clock <= that clock is in them);
4. **pull**   — every owner's latest published shard into its local copy, waiting only
   until each owner's applied-through clock is >= t - 2s.

So no rank runs more than ``s`` steps ahead of another.  The staleness of a step is its
clock minus the applied-through clock of the parameters it pulled (the oldest of its own
shard's and every pulled shard's): the own shard holds every push through t - s and every
pulled shard every push through t - 2s, so **max_staleness <= 2s** — the one bound the
docstring, the kernel's measurement (``async_ps.hip``) and the tests all state.  (The
gradient of the NEXT clock, t + 1, is computed on those parameters.)  s = 0 is lockstep
(each rank's push still applied separately).  Staleness is bounded and measured, never
zero-by-barrier.  At the end ``finish()`` drains: every owner applies every push
and every rank pulls the final shards, so replicas agree.

Two transports implement the protocol:
* ``AsyncPSGloo`` — torch.distributed point-to-point (gloo, CPU): the emulation used by the
  CPU tests and the eager program;
* ``AsyncPSDevice`` (``async_ps.hip``) — IPC-mapped peer buffers over xGMI, ONE kernel
  launch per step with device-side clocks and bounded waits (``parallel.xgmi`` rules).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import optim_ref
from .xgmi import _line_up, max_blocks_from_env, pool_get, pool_put

GRAD, PARAM = 0, 1


def staleness_from(cfg) -> int:
    """``options.staleness`` of the job config (default CSA_STALENESS or 2)."""
    raw = getattr(cfg, "raw", None) or {}
    opts = raw.get("options", {}) if isinstance(raw, dict) else {}
    if isinstance(opts, dict) and "staleness" in opts:
        return max(0, int(opts["staleness"]))
    return int(os.environ.get("CSA_STALENESS", "2"))


def _tag(kind: int, clock: int) -> int:
    return 2 * clock + kind


class AsyncPSGloo:
    """The protocol over torch.distributed isend / irecv (CPU tensors, gloo)."""

    def __init__(self, rank: int, world: int, shard: int, staleness: int, opt_id: int, lr: float):
        self.r, self.W, self.sh, self.s = rank, world, shard, staleness
        self.opt_id, self.lr = opt_id, lr
        self.next_apply = (0, 0)                  # (clock, source) of the next push to apply
        self.applied = 0                          # pushes applied (Adam's 1-based t)
        self.grad_recv: Dict[Tuple[int, int], Tuple[object, torch.Tensor]] = {}
        self.own: Dict[int, torch.Tensor] = {}    # my own push per clock (never leaves the rank)
        self.sends: List[object] = []
        # params from each owner: posted receive for its next publication, latest received
        self.par_req: Dict[int, Tuple[object, torch.Tensor]] = {}
        self.par_clock = {p: -1 for p in range(world)}      # next publication index expected
        self.par_at = {p: -1 for p in range(world)}         # owner's applied-through clock
        self.par_final = {p: False for p in range(world)}
        self.max_staleness = 0
        self.t = 0

    # ---- helpers ----
    def _lo(self, p: int) -> int:
        return p * self.sh

    def _post_grad(self, c: int, q: int) -> None:
        if (c, q) not in self.grad_recv:
            buf = torch.empty(self.sh)
            self.grad_recv[(c, q)] = (dist.irecv(buf, src=q, tag=_tag(GRAD, c)), buf)

    def _post_param(self, p: int) -> None:
        if p not in self.par_req and not self.par_final[p]:
            buf = torch.empty(self.sh + 2)
            self.par_clock[p] += 1
            self.par_req[p] = (dist.irecv(buf, src=p, tag=_tag(PARAM, self.par_clock[p])), buf)

    def _apply(self, w: torch.Tensor, slots: torch.Tensor, g: torch.Tensor) -> None:
        self.applied += 1
        optim_ref.step_ref(self.opt_id, w, g, slots, self.lr, self.applied)

    def applied_through(self) -> int:
        c, q = self.next_apply
        return c - 1

    def _apply_arrived(self, w, slots, t: int, must: int) -> None:
        """Apply pushes in (clock, source) order up to clock t: blocking for clocks <= must."""
        while True:
            c, q = self.next_apply
            if c > t:
                return
            if q == self.r:
                g = self.own.pop(c)
            else:
                self._post_grad(c, q)
                req, buf = self.grad_recv[(c, q)]
                if c > must and not req.is_completed():
                    return
                req.wait()
                del self.grad_recv[(c, q)]
                g = buf
            self._apply(w, slots, g)
            self.next_apply = (c, q + 1) if q + 1 < self.W else (c + 1, 0)

    def _publish(self, w: torch.Tensor, final: bool) -> None:
        msg = torch.empty(self.sh + 2)
        msg[0] = float(self.applied_through())
        msg[1] = 1.0 if final else 0.0
        msg[2:] = w
        for p in range(self.W):
            if p != self.r:
                self.sends.append((dist.isend(msg, dst=p, tag=_tag(PARAM, self.t)), msg))
        self.sends = [x for x in self.sends if not x[0].is_completed()]

    def _pull(self, flat: torch.Tensor, need: int) -> None:
        for p in range(self.W):
            if p == self.r:
                continue
            while True:
                self._post_param(p)
                if p not in self.par_req:
                    break                                   # owner published its final shard
                req, buf = self.par_req[p]
                if self.par_at[p] >= need and not req.is_completed():
                    break
                req.wait()
                del self.par_req[p]
                self.par_at[p] = int(buf[0].item())
                self.par_final[p] = buf[1].item() > 0
                flat[self._lo(p):self._lo(p) + self.sh].copy_(buf[2:])

    # ---- the step ----
    def step(self, flat_grad: torch.Tensor, flat: torch.Tensor, slots: torch.Tensor) -> None:
        t, s = self.t, self.s
        for p in range(self.W):
            gp = flat_grad[self._lo(p):self._lo(p) + self.sh]
            if p == self.r:
                self.own[t] = gp.clone()
            else:
                buf = gp.clone()
                self.sends.append((dist.isend(buf, dst=p, tag=_tag(GRAD, t)), buf))
        w = flat[self._lo(self.r):self._lo(self.r) + self.sh]
        self._apply_arrived(w, slots, t, t - s)
        self._publish(w, final=False)
        self._pull(flat, t - 2 * s)
        at = min([self.applied_through()] + [self.par_at[p] for p in range(self.W) if p != self.r])
        self.max_staleness = max(self.max_staleness, t - at)
        self.t += 1

    def finish(self, flat: torch.Tensor, slots: torch.Tensor) -> None:
        """Apply every outstanding push, publish the final shard, pull every final shard."""
        last = self.t - 1
        w = flat[self._lo(self.r):self._lo(self.r) + self.sh]
        self._apply_arrived(w, slots, last, last)
        self._publish(w, final=True)
        self._pull(flat, last)
        for p in range(self.W):                  # through each owner's final publication
            while p != self.r and not self.par_final[p]:
                self._pull(flat, self.par_at[p] + 1)
        for work, _ in self.sends:
            work.wait()
        self.sends = []


class AsyncPSDevice:
    """The protocol on the GPU: IPC-mapped uncached peer buffers (inbox ring, arrival flags,
    double-buffered seqlocked outbox) and ONE ``aps_kernel`` launch per step
    (csrc/comm/async_ps.hip), capturable in the step's HIP graph."""

    def __init__(self, rank: int, world: int, shard: int, staleness: int, opt_id: int, lr: float,
                 device: torch.device, group=None, timeout_s: Optional[float] = None):
        from ..ops import fused as K
        if shard % 4:
            raise ValueError("async_ps: the shard must be a multiple of 4 floats")
        self.lib = K.load(required=True)
        self.r, self.W, self.sh, self.s = rank, world, shard, staleness
        self.opt_id, self.lr, self.device = opt_id, lr, device
        self.R = 2 * staleness + 2
        # every workgroup of a step waits on its peers' (bounded): CSA_XGMI_BLOCKS caps them
        # so ranks sharing one GPU keep all their workgroups resident (parallel/xgmi.py)
        # (chunks of >= 4096 floats; up to 512 of them: two workgroups per CU, each thread
        # with few enough float4 rounds that the chunk is not a chain of load latencies)
        self.nb = max(1, min(512, (shard + 4095) // 4096))
        cap = max_blocks_from_env()
        if cap:
            self.nb = max(1, min(self.nb, cap))
        self.timeout_s = timeout_s if timeout_s is not None else float(os.environ.get("CSA_XGMI_TIMEOUT_S", "20"))
        sizes = [self.R * world * shard * 4, self.R * world * self.nb * 4, 2 * shard * 4, 2 * self.nb * 4,
                 2 * self.nb * 4]
        hb = self.lib.csa_xgmi_handle_bytes()
        self._dev = device.index if device.index is not None else torch.cuda.current_device()
        self._local: List[int] = []
        self._local_n: List[int] = []
        self._opened: List[int] = []
        handles: Optional[List[bytes]] = []
        with torch.cuda.device(device):
            try:
                for n in sizes:
                    ptr, h = pool_get(self.lib, self._dev, n)      # recycled, never hipFree'd
                    self._local.append(ptr)
                    self._local_n.append(n)
                    handles.append(h)
            except Exception:
                handles = None
            allh: List[Optional[List[bytes]]] = [None] * world
            dist.all_gather_object(allh, handles, group=group)
            if any(h is None for h in allh):
                self.close(barrier=False)
                raise RuntimeError("async_ps: a rank could not allocate its peer buffers")
            ptrs: List[int] = []
            ok = True
            for q in range(world):
                for k in range(5):
                    if q == rank:
                        ptrs.append(self._local[k])
                        continue
                    p = C.c_void_p()
                    if self.lib.csa_xgmi_open(C.create_string_buffer(allh[q][k], hb), C.byref(p)):
                        ok = False
                        ptrs.append(0)
                        continue
                    self._opened.append(p.value)
                    ptrs.append(p.value)
            oks: List[Optional[bool]] = [None] * world
            dist.all_gather_object(oks, ok, group=group)
            if not all(oks):
                self.close(barrier=False)
                raise RuntimeError("async_ps: mapping a peer buffer failed")
        self._bufs = (C.c_void_p * (5 * world))(*ptrs)
        # per workgroup: next clock, next source, pushes applied, clock t, max staleness
        self.prog = torch.zeros(5 * self.nb, dtype=torch.int32, device=device)
        self.state = torch.zeros(4, dtype=torch.int32, device=device)     # -, -, err
        # my own pushes not applied in their own launch: local (cached) memory, never mapped
        self.selfbox = torch.zeros(self.R * shard, dtype=torch.float32, device=device)
        self.group = group

    def reset(self) -> None:
        """Collective: back to clock 0 with empty mailboxes (after the engine's throw-away
        warm-up steps restored the model state)."""
        torch.cuda.synchronize(self.device)
        if dist.is_initialized():
            _line_up(self.group, self.device)
        nbytes = [self.R * self.W * self.nb * 4, 2 * self.nb * 4, 2 * self.nb * 4]
        ptrs = [self._local[1], self._local[3], self._local[4]]
        self.lib.csa_zero((C.c_void_p * 3)(*ptrs), (C.c_long * 3)(*[n // 4 for n in nbytes]), 3,
                          torch.cuda.current_stream(self.device).cuda_stream)
        self.prog.zero_(); self.state.zero_()
        torch.cuda.synchronize(self.device)
        if dist.is_initialized():
            _line_up(self.group, self.device)

    def _launch(self, flat_grad, flat, slots, drain: int) -> None:
        s0 = slots[0, :] if slots.shape[0] > 0 else None
        s1 = slots[1, :] if slots.shape[0] > 1 else None
        rc = self.lib.csa_aps_step(
            self.r, self.W, self.R, self.s, self.sh, self.nb, self._bufs, flat_grad.data_ptr(), flat.data_ptr(),
            None if s0 is None else s0.data_ptr(), None if s1 is None else s1.data_ptr(),
            self.selfbox.data_ptr(), self.opt_id,
            float(self.lr), self.prog.data_ptr(), self.state.data_ptr(), drain,
            self.timeout_s, torch.cuda.current_stream(self.device).cuda_stream)
        if rc:
            raise RuntimeError(f"async_ps step launch failed ({rc})")

    def step(self, flat_grad: torch.Tensor, flat: torch.Tensor, slots: torch.Tensor) -> None:
        self._launch(flat_grad, flat, slots, 0)

    def finish(self, flat: torch.Tensor, slots: torch.Tensor) -> None:
        self._launch(flat, flat, slots, 1)             # (the gradient is not read when draining)
        torch.cuda.synchronize(self.device)
        # (no local raise: TrainEngine.finish_async agrees on the error across ranks)

    def error(self) -> int:
        return int(self.state[2].item())

    def check(self) -> None:
        if self.error():
            raise RuntimeError("async_ps: a peer wait timed out (state poisoned)")

    @property
    def max_staleness(self) -> int:
        return int(self.prog.view(-1, 5)[:, 4].max().item())

    @property
    def applied(self) -> int:
        """Pushes applied to EVERY chunk of this owner's shard (the slowest workgroup's count)."""
        return int(self.prog.view(-1, 5)[:, 2].min().item())

    @property
    def t(self) -> int:
        return int(self.prog.view(-1, 5)[:, 3].min().item())

    def close(self, barrier: bool = True) -> None:
        """Collective: every rank's kernels drain before any buffer is freed."""
        if not self._local and not self._opened:
            return
        torch.cuda.synchronize(self.device)
        if barrier and dist.is_initialized():
            _line_up(self.group, self.device)
        for p in self._opened:
            self.lib.csa_xgmi_close(p)
        for p, n in zip(self._local, self._local_n):       # back to the process pool
            pool_put(self._dev, p, n)
        self._local, self._local_n, self._opened = [], [], []


def make_async_ps(eng, lo: int, hi: int):
    """The transport for this engine: IPC peer buffers on a GPU, gloo point-to-point on CPU."""
    from .dist import DistContext  # noqa: F401  (documented dependency)
    s = staleness_from(eng.cfg)
    ctx = eng.ctx
    if eng.device.type == "cuda":
        return AsyncPSDevice(ctx.rank, ctx.world, hi - lo, s, eng.opt_id, eng.lr, eng.device)
    return AsyncPSGloo(ctx.rank, ctx.world, hi - lo, s, eng.opt_id, eng.lr)

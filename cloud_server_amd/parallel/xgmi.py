"""Peer-buffer collectives over xGMI (the custom one-shot path of SURVEY.md §5.8).

Each ``XgmiChannel`` owns, per rank, an uncached receive buffer ``[2][world][slot]``
and a flag array, both exported with ``hipIpcGetMemHandle`` and mapped into every
other rank with ``hipIpcOpenMemHandle`` (handles travel through the process group's
object all-gather; the data plane never touches RCCL).  A call is ONE kernel launch
(``csrc/comm/xgmi.hip``): every rank pushes its message to all peers over its 7 xGMI
links at once and each block then waits only on the flags of its own chunk.  The epoch
counter lives on the device, so a call captured into a HIP graph replays correctly.

Reference: the per-step variable pull / gradient push between worker and PS over TF
gRPC (construct_distribute.py:355-357, 413).

Rules
* one channel = one device-ordered sequence of calls; call sites that can run on
  different streams concurrently get different channels (``XgmiComm.channel(tag)``);
* every rank must issue the same calls on a channel in the same order (SPMD);
* waits are bounded (``timeout_s``): a missing peer sets the channel's error word and
  later calls return at once; ``check()`` turns it into an exception on the host.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import fused as K

OP_GATHER, OP_ALLREDUCE, OP_ALLREDUCE_2SHOT = 0, 1, 2
# default protocol crossover (per-rank message bytes) until the start-up tuner measured
# both on the real links: one-shot below (one flag round trip), two-shot above (2 (W-1)/W
# of the message leaves each GPU instead of (W-1) x)
TWO_SHOT_MIN_BYTES = 256 * 1024


def _line_up(group, device) -> None:
    """Every rank reaches this point before any goes on: a 1-element all-reduce waited on
    by the host (the collective the tuner already uses to line ranks up; a ``dist.barrier``
    here was followed by a process abort in the next test's graph capture under RCCL)."""
    t = torch.zeros(1, device=device)
    dist.all_reduce(t, group=group)
    t.item()


def _aligned(t: torch.Tensor) -> bool:
    return t.is_contiguous() and t.data_ptr() % 16 == 0 and (t.numel() * t.element_size()) % 16 == 0


# Peer buffers are recycled inside the process, never freed before exit: after a hipFree an
# uncached allocation of the same size can come back at the same address while a peer's
# mapping of the old one is stale (a third channel set created in one process timed out
# with one rank never seeing the other's pushes: profiles/r4_notes.md).  Keyed by
# (device index, bytes).
_POOL: Dict[Tuple[int, int], List[int]] = {}


def pool_get(lib, dev: int, nbytes: int) -> Tuple[int, bytes]:
    """A zeroed uncached peer buffer of ``nbytes`` on device ``dev`` (from the process pool
    when one is free) and its freshly exported IPC handle."""
    h = C.create_string_buffer(lib.csa_xgmi_handle_bytes())
    free = _POOL.get((dev, nbytes))
    if free:
        ptr = free.pop()
        rc = lib.csa_xgmi_reuse(C.c_void_p(ptr), nbytes, h)
        if rc:
            raise RuntimeError(f"xgmi buffer reuse failed ({rc})")
        return ptr, h.raw
    p = C.c_void_p()
    rc = lib.csa_xgmi_alloc(nbytes, C.byref(p), h)
    if rc:
        raise RuntimeError(f"xgmi alloc failed ({rc})")
    return p.value, h.raw


def pool_put(dev: int, ptr: int, nbytes: int) -> None:
    """Back to the process pool (never hipFree'd while a peer may still map it)."""
    _POOL.setdefault((dev, nbytes), []).append(ptr)


class XgmiChannel:
    def __init__(self, rank: int, world: int, slot_bytes: int, device: torch.device,
                 group=None, timeout_s: float = 20.0):
        if not 1 <= world <= 8:
            raise ValueError("xGMI channel: 1..8 ranks of one node")
        self.lib = K.load(required=True)
        self.rank, self.world, self.device = rank, world, device
        self.slot_bytes = (int(slot_bytes) + 15) // 16 * 16
        self.timeout_s = timeout_s
        hb = self.lib.csa_xgmi_handle_bytes()
        nblk = self.lib.csa_xgmi_max_blocks()
        # receive slots (+ slack: two-shot shards round up to 16 B) and per-phase flags
        sizes = (2 * world * self.slot_bytes + 64 * world, 2 * 2 * nblk * 8 * 4)
        self._local: List[int] = []
        self._local_n: List[int] = []
        self._opened: List[int] = []
        self._dev = device.index if device.index is not None else torch.cuda.current_device()
        # every failure is agreed on collectively (all ranks raise together), so a rank
        # that cannot allocate or map never leaves its peers inside a collective
        handles: Optional[List[bytes]] = []
        with torch.cuda.device(device):
            try:
                for n in sizes:
                    ptr, h = pool_get(self.lib, self._dev, n)
                    self._local.append(ptr)
                    self._local_n.append(n)
                    handles.append(h)
            except Exception:
                handles = None
            allh: List[Optional[List[bytes]]] = [None] * world
            dist.all_gather_object(allh, handles, group=group)
            if any(h is None for h in allh):
                self.close()
                raise RuntimeError("xgmi: a rank could not allocate its peer buffers")
            ptrs: List[List[int]] = [[], []]
            ok = True
            for r in range(world):
                for k in range(2):
                    if r == rank:
                        ptrs[k].append(self._local[k])
                        continue
                    p = C.c_void_p()
                    rc = self.lib.csa_xgmi_open(C.create_string_buffer(allh[r][k], hb), C.byref(p))
                    if rc:
                        ok = False
                        ptrs[k].append(0)
                        continue
                    self._opened.append(p.value)
                    ptrs[k].append(p.value)
            oks: List[Optional[bool]] = [None] * world
            dist.all_gather_object(oks, ok, group=group)
            if not all(oks):
                self.close()
                raise RuntimeError(f"xgmi: mapping a peer buffer failed on rank(s) "
                                   f"{[r for r, o in enumerate(oks) if not o]}")
        self._bufs = (C.c_void_p * world)(*ptrs[0])
        self._flags = (C.c_void_p * world)(*ptrs[1])
        self.state = torch.zeros(4, dtype=torch.int32, device=device)   # seq, done, err, pad
        # per-block record of the last call (csrc/comm/xgmi.hip XgArgs::diag), read by
        # ``diag()`` after a timeout
        self._dw = self.lib.csa_xgmi_diag_words()
        self.diag_buf = torch.zeros(nblk * self._dw, dtype=torch.int64, device=device)
        # workgroups per call (0: one per ~8 KB of the per-rank message, at most 256)
        self.nblocks = 0
        # upper bound on workgroups per call (CSA_XGMI_BLOCKS; 0 = none).  Every block of a
        # call waits on its peers' blocks, so all ranks' blocks of a call must be resident
        # at once: ranks that share ONE GPU (the one-GPU multi-process tests) split its
        # ~1280 slots for 256-thread blocks between them; on a node each rank owns a GPU
        self.max_blocks = max_blocks_from_env()
        # all-reduce protocol: None = by size (TWO_SHOT_MIN_BYTES); the tuner pins it
        self.protocol: Optional[str] = None

    # ---------------------------------------------------------------- calls
    def blocks_for(self, nbytes: int) -> int:
        """Workgroups of a call moving ``nbytes`` per rank (0 = the kernel's own choice)."""
        nb = self.nblocks
        if self.max_blocks > 0:
            nb = min(nb if nb > 0 else max(1, (nbytes // 16 + 511) // 512), self.max_blocks)
        return nb

    def _run(self, op: int, srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor]) -> None:
        n = len(srcs)
        sb = [s.numel() * s.element_size() for s in srcs]
        rc = self.lib.csa_xgmi_run(
            op, self.rank, self.world, self.slot_bytes, self._bufs, self._flags, n,
            (C.c_void_p * n)(*[s.data_ptr() for s in srcs]), (C.c_void_p * n)(*[d.data_ptr() for d in dsts]),
            (C.c_long * n)(*sb), self.state.data_ptr(), self.timeout_s, self.blocks_for(sum(sb)),
            self.diag_buf.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        if rc:
            raise RuntimeError(f"xgmi collective launch failed ({rc})")

    def all_gather(self, pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> None:
        """``out`` = rank-major concatenation of every rank's ``local`` (per pair)."""
        self._run(OP_GATHER, [p[0] for p in pairs], [p[1] for p in pairs])

    def all_reduce(self, tensors: Sequence[torch.Tensor], protocol: Optional[str] = None) -> None:
        """In-place fp32 SUM over ranks (identical bits on every rank: fixed rank order).
        ``protocol``: "oneshot" (push everything to everyone), "twoshot" (reduce-scatter +
        all-gather), default the channel's pinned choice or the size crossover."""
        p = protocol or self.protocol
        if self.world == 1:
            p = "oneshot"             # nothing to scatter (and no room for two phases)
        if p is None:
            nbytes = sum(t.numel() * t.element_size() for t in tensors)
            p = "twoshot" if nbytes >= TWO_SHOT_MIN_BYTES and self.world > 2 else "oneshot"
        self._run(OP_ALLREDUCE_2SHOT if p == "twoshot" else OP_ALLREDUCE, tensors, tensors)

    def reduce_scatter_range(self, flat: torch.Tensor, lo: int, hi: int, shard: int,
                             shard_out: torch.Tensor) -> None:
        """Elements [lo, hi) of the flat fp32 buffer, summed over ranks into their OWNERS
        (element i belongs to rank i // shard): this rank's part of the range lands in
        ``shard_out[i - rank * shard]``.  Every element leaves its GPU at most once."""
        rc = self.lib.csa_xgmi_reduce_scatter(
            self.rank, self.world, self.slot_bytes, self._bufs, self._flags, flat.data_ptr(), lo * 4,
            (hi - lo) * 4, shard * 4, shard_out.data_ptr(), self.state.data_ptr(), self.timeout_s,
            self.blocks_for((hi - lo) * 4), self.diag_buf.data_ptr(),
            torch.cuda.current_stream(self.device).cuda_stream)
        if rc:
            raise RuntimeError(f"xgmi reduce-scatter launch failed ({rc})")

    def fits(self, tensors: Sequence[torch.Tensor]) -> bool:
        return (len(tensors) <= 8 and all(_aligned(t) for t in tensors)
                and sum(t.numel() * t.element_size() for t in tensors) <= self.slot_bytes)

    def error(self) -> int:
        return int(self.state[2].item())

    def diag(self) -> List[dict]:
        """Per-block record of the LAST call on this channel (synchronises the device):
        epoch, wall-clock stamps (device-wide 100 MHz clock), status and — for a block
        that timed out — the missing source, the flag value it last saw and that source's
        own copy of the flag.  Blocks that did not take part in the last call are skipped."""
        torch.cuda.synchronize(self.device)
        d = self.diag_buf.view(-1, self._dw).cpu().tolist()
        out = []
        for b, (e, t0, tp, tw, stt, src, seen, own) in enumerate(d):
            if t0 == 0:
                continue
            rec = {"block": b, "epoch": e, "t_start": t0, "t_pub": tp, "t_wait": tw,
                   "status": {0: "running", 1: "ok", 2: "timeout"}.get(stt, stt)}
            if stt == 2:
                rec.update(missing=src, seen=seen, src_own_copy=own)
            out.append(rec)
        return out

    def diag_summary(self) -> dict:
        """Compact form of ``diag()`` for failure messages: the epochs blocks used, the
        start / publish window, and every timed-out block's record."""
        recs = self.diag()
        if not recs:
            return {"blocks": 0}
        starts = [r["t_start"] for r in recs]
        pubs = [r["t_pub"] for r in recs if r["t_pub"]]
        return {"blocks": len(recs), "epochs": sorted({r["epoch"] for r in recs}),
                "t_start": [min(starts), max(starts)], "t_pub": [min(pubs), max(pubs)] if pubs else None,
                "unpublished": [r["block"] for r in recs if not r["t_pub"]][:16],
                "timeouts": [r for r in recs if r["status"] == "timeout"][:8],
                "state": self.state.tolist()}

    def check(self) -> None:
        if self.error():
            raise RuntimeError("xGMI collective timed out waiting for a peer (channel poisoned)")

    def close(self) -> None:
        if not self._local and not self._opened:
            return
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.lib.csa_xgmi_close(p)
        for p, n in zip(self._local, self._local_n):       # back to the process pool
            pool_put(self._dev, p, n)
        self._local, self._local_n, self._opened = [], [], []


class XgmiComm:
    """Channels by call-site tag, created lazily (collectively) on first use — which must
    happen outside HIP-graph capture (the engine's eager warm-up steps do it)."""

    def __init__(self, rank: int, world: int, device: torch.device, group=None, timeout_s: Optional[float] = None):
        self.rank, self.world, self.device, self.group = rank, world, device, group
        # bound of every peer wait (CSA_XGMI_TIMEOUT_S, default 20 s): a missing peer
        # poisons the channel instead of hanging the GPU
        self.timeout_s = timeout_s if timeout_s is not None else float(os.environ.get("CSA_XGMI_TIMEOUT_S", "20"))
        self.channels: Dict[str, XgmiChannel] = {}

    def channel(self, tag: str, nbytes: int) -> XgmiChannel:
        ch = self.channels.get(tag)
        if ch is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"xgmi channel {tag!r} first used inside graph capture")
            ch = XgmiChannel(self.rank, self.world, nbytes, self.device, self.group, self.timeout_s)
            self.channels[tag] = ch
        return ch

    def check(self) -> None:
        for ch in self.channels.values():
            ch.check()

    def close(self) -> None:
        """Collective (every rank calls it): a rank frees its buffers only once EVERY rank's
        last call has drained — a peer still running would otherwise write through its
        mapping into memory this rank has freed, and the allocator may already have handed
        those bytes to a new channel (whose flags then read stale epochs)."""
        if not self.channels:
            return
        torch.cuda.synchronize(self.device)
        if dist.is_initialized():
            _line_up(self.group, self.device)
        for ch in self.channels.values():
            ch.close()
        self.channels.clear()


def self_test(comm: XgmiComm) -> bool:
    """Collective sanity check run once at start-up: an all-gather and an all-reduce of
    rank-dependent data, verified on the host; every rank learns whether ALL passed."""
    dev = comm.device
    ok = True
    # every rank loads the kernel library's code object BEFORE any rank launches a waiting
    # kernel: a rank still loading it (seconds, with several processes starting at once)
    # would otherwise leave its peers' bounded waits to time out
    lib = K.load(required=True)
    z = torch.zeros(4, device=dev)
    lib.csa_zero((C.c_void_p * 1)(z.data_ptr()), (C.c_long * 1)(4), 1, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    _line_up(comm.group, dev)
    ch = None
    try:
        W, r = comm.world, comm.rank
        x = torch.arange(1024, dtype=torch.float32, device=dev) + 1000.0 * r
        out = torch.empty(W * 1024, dtype=torch.float32, device=dev)
        ch = XgmiChannel(comm.rank, W, 4096, dev, comm.group, timeout_s=20.0)
        ch.all_gather([(x, out)])
        want = torch.cat([torch.arange(1024, dtype=torch.float32, device=dev) + 1000.0 * k for k in range(W)])
        y = x.clone()
        ch.all_reduce([y], protocol="oneshot")
        y2 = x.clone()
        ch.all_reduce([y2], protocol="twoshot" if W > 2 else "oneshot")
        torch.cuda.synchronize(dev)
        want_sum = W * torch.arange(1024, dtype=torch.float32, device=dev) + 1000.0 * sum(range(W))
        checks = {"timeout": ch.error() == 0, "gather": torch.equal(out, want),
                  "oneshot": torch.equal(y, want_sum), "twoshot": torch.equal(y2, want_sum)}
        ok = all(checks.values())
        if not ok:
            comm.self_test_reason = "failed: " + ",".join(k for k, v in checks.items() if not v)
    except Exception as exc:
        ok = False
        comm.self_test_reason = f"{type(exc).__name__}: {exc}"
    torch.cuda.synchronize(dev)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=comm.group)
    passed = bool(flag.item())       # every rank's kernels have drained: safe to free
    if ch is not None:
        ch.close()
    return passed


def max_blocks_from_env() -> int:
    """``CSA_XGMI_BLOCKS``: cap on the workgroups of one peer-buffer call (0 / unset: none)."""
    try:
        return max(0, int(os.environ.get("CSA_XGMI_BLOCKS", "0")))
    except ValueError:
        return 0


def shared_gpu_block_cap(world: int, live_channels: int = 1) -> int:
    """The ``CSA_XGMI_BLOCKS`` that lets ``world`` ranks sharing ONE GPU keep every block of
    ``live_channels`` concurrent calls resident: half of the chip's ~1280 slots for 256-
    thread blocks (5 per CU at the kernels' register budget), the other half left to the
    ranks' own compute kernels running beside them."""
    return max(8, 640 // (world * max(1, live_channels)) // 8 * 8)


def enabled_by_env() -> str:
    """``CSA_XGMI``: ``auto`` (default: on for RCCL jobs after a passing self-test),
    ``1`` (on, fail loudly), ``0`` (RCCL only)."""
    return os.environ.get("CSA_XGMI", "auto").lower()

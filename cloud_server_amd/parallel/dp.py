"""Data-parallel gradient synchronisation strategies over RCCL/xGMI.

Reference: asynchronous between-graph replication through a parameter server —
``replica_device_setter`` puts every variable on ``/job:ps`` and each worker pulls
vars / pushes grads over gRPC per ``sess.run`` (construct_distribute.py:355-357, 413;
SURVEY.md §2.3).  On one MI355X node that becomes:

* ``allreduce`` (default) — synchronous DP: every rank holds the params; the flat fp32
  gradient buffer is summed with RCCL all-reduce in a few large buckets (xGMI ring
  collectives are per-link bound, so few large messages beat many small ones).  The
  1/world averaging factor is folded into the loss-gradient seed, so the all-reduced
  SUM is already the mean and no extra scaling pass is needed.
* ``ps`` — the parameter-server capability, sharded and synchronous (ZeRO-1 style):
  reduce-scatter gradients to each rank's owned shard, the owner applies the fused
  optimizer to its shard only (optimizer slots exist only for the shard, the PS
  analogue of accumulators living on ``/job:ps``), then all-gather the new params.
* ``lowrank`` — exact sync DP for the dense layers at small per-rank batch: a dense
  weight gradient is ``Xᵀ·dY`` with K = per-rank batch, so instead of all-reducing the
  [in, out] gradient we all-gather the [B, in] activations and [B, out] output grads
  and every rank forms the global ``Xᵀ·dY`` locally (K = world·B).  For the sample
  config fc1 that is 0.9 MB gathered per rank instead of an 8 MB all-reduce.

All strategies are written against ``torch.distributed`` so the identical code runs on
gloo (CPU tests) and RCCL (MI355X).  On a single node with RCCL the latency-bound
collectives (lowrank gathers, the remainder all-reduce, allreduce buckets) go through
the xGMI peer-buffer path (``parallel.xgmi``, one launch, all 7 links) instead, once a
start-up self-test passed on every rank (``CSA_XGMI=auto|1|0``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..utils.tracing import trace_range
from .dist import DistContext
from . import xgmi as _xg
from ..utils.graphs import capture, wait_retired

DEFAULT_BUCKET_BYTES = 32 << 20   # one bucket covers the sample model's 9.1 MB gradient


_CAP: list = []        # [(default group, capture group, retired)] of this process


def capture_group(device: torch.device):
    """The process's dedicated capture group over all ranks (``GradSync._setup_capture_
    group``), created collectively on first use per default group — every GradSync (each
    engine, the strategy tuner's trial engines) shares it — with its connection check
    retired by the watchdog before any capture uses it.  Returns (group, retired)."""
    default = dist.distributed_c10d._get_default_group()
    if _CAP and _CAP[0][0] is default:
        return _CAP[0][1], _CAP[0][2]
    # its RCCL stream from torch's HIGH-priority stream pool: the default group draws from
    # the low-priority one, so the two groups can never share a HIP stream (a captured
    # collective would otherwise turn the default group's stream into a capturing one under
    # an eager work the watchdog still polls: hipErrorCapturedEvent, utils/streams.py)
    opts = None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
    except Exception:  # pragma: no cover - backend without options
        opts = None
    g = dist.new_group(backend="nccl", device_id=device, pg_options=opts)
    t = torch.ones(1, device=device)
    dist.all_reduce(t, group=g)
    if int(t.item()) != dist.get_world_size():
        raise RuntimeError("capture process group: connection check failed")
    retired = wait_retired(g)
    _CAP[:] = [(default, g, retired)]
    return g, retired


class GradSync:
    def __init__(self, ctx: DistContext, numel: int, strategy: str = "allreduce",
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES):
        if strategy not in ("allreduce", "ps", "lowrank", "async_ps"):
            raise ValueError(f"unknown DP strategy {strategy!r}")
        self.ctx, self.numel, self.strategy = ctx, numel, strategy
        # parameters / optimizer slots sharded over owner ranks (the PS placement)
        self.sharded = strategy in ("ps", "async_ps") and ctx.enabled
        if self.sharded and numel % ctx.world:
            raise ValueError(f"{strategy} strategy needs the flat buffer padded to a multiple of world")
        self.shard = numel // ctx.world if ctx.enabled else numel
        self.bucket_elems = max(1, bucket_bytes // 4)
        # (grouped RCCL launches for the multi-tensor collectives are not used: a grouped
        # collective inside HIP-graph capture crashed capture_end on ROCm 7 / torch 2.10)
        self.xgmi: Optional[_xg.XgmiComm] = None
        self.xgmi_reason = "off"
        self.xgmi_mode = _xg.enabled_by_env()
        self.xgmi_tuning: dict = {}      # tag -> {"bytes", "xgmi_us", "rccl_us"} (auto mode)
        self._choice: dict = {}
        self.timing: Optional[list] = None   # set by TrainEngine.probe: (start, end) events per call
        # further poisoned-transport probes (the async_ps device state): () -> nonzero on error
        self.extra_errors: List = []
        # CSA_DETERMINISTIC=1: every SUM is formed in a fixed rank order — the
        # xGMI kernels (one-/two-shot, range reduce-scatter: fixed-order by construction),
        # or, where they do not apply, an exact all-gather followed by a rank-ordered fold.
        # Bitwise-repeatable and identical on every rank; never RCCL's reductions.
        self.det = os.environ.get("CSA_DETERMINISTIC", "0") == "1"
        self.cap_group = None
        self._setup_capture_group()
        self._setup_xgmi()

    # ---- RCCL: captured collectives on their own communicator ----
    def _setup_capture_group(self) -> None:
        """RCCL collectives captured into HIP graphs run on a DEDICATED process group.

        The process-group watchdog polls the end event of every EAGER collective until it
        reaps it; a capture that contains a collective pulls that group's internal RCCL
        stream into the capture, and querying an event recorded on a stream that is
        capturing aborts the process (hipErrorCapturedEvent — round 4's intermittent
        suite abort, profiles/r4_notes.md).  So eager collectives (warm-up steps, the
        tuner's warm-up, agreement flags) stay on the default group and every collective
        issued while capturing goes to ``cap_group`` (``_pg``), whose stream therefore never
        carries an eager event the watchdog is still polling.  The group's communicator is
        connected eagerly (``device_id``; ``NCCL_RUNTIME_CONNECT=0`` from
        ``init_distributed`` sets every connection up at creation), and its ONE eager
        collective — a connection check — is waited on until the watchdog has RETIRED it
        (the flight recorder's active list, an observable condition, not a timed sleep)."""
        if not (self.ctx.enabled and self.ctx.backend == "nccl" and dist.is_available() and dist.is_initialized()):
            return
        if dist.get_backend() != "nccl":
            return                   # (the one-GPU multi-process tests: a gloo group, no RCCL)
        if os.environ.get("CSA_CAPTURE_GROUP", "1") != "1":
            return
        self.cap_group, self.cap_group_retired = capture_group(self.ctx.device)

    def _pg(self):
        """The process group of a data-plane collective issued now: the capture group while
        the current stream is capturing, else the default group."""
        if self.cap_group is not None and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return self.cap_group
        return None

    @contextlib.contextmanager
    def _timed(self):
        """Bracket one collective with timing events on the current stream when a probe
        step asked for it (never inside graph capture)."""
        if self.timing is None or not self.ctx.device.type == "cuda" or torch.cuda.is_current_stream_capturing():
            with trace_range("csa.comm"):
                yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        with trace_range("csa.comm"):
            yield
        b.record()
        self.timing.append((a, b))

    def _setup_xgmi(self) -> None:
        mode = self.xgmi_mode
        if self.strategy == "async_ps":
            self.xgmi_reason = "async_ps: its own peer-buffer transport"
            return
        if mode in ("0", "off", "false") or self.ctx.backend != "nccl" or not self.ctx.enabled:
            self.xgmi_reason = "disabled" if self.ctx.enabled else "single rank"
            return
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.ctx.world)))
        if local_world != self.ctx.world or self.ctx.world > 8:
            self.xgmi_reason = "multi-node job: RCCL"
            return
        comm = _xg.XgmiComm(self.ctx.rank, self.ctx.world, self.ctx.device)
        if _xg.self_test(comm):
            self.xgmi, self.xgmi_reason = comm, "on"
            return
        comm.close()
        if mode in ("1", "on", "true"):
            raise RuntimeError("CSA_XGMI=1 but the xGMI peer-buffer self-test failed (rank "
                               f"{self.ctx.rank}: {getattr(comm, 'self_test_reason', 'another rank failed')})")
        self.xgmi_reason = "self-test failed: RCCL"

    def check(self) -> None:
        """Raise if a peer-buffer collective timed out (its results are not valid)."""
        if self.xgmi is not None:
            self.xgmi.check()

    def check_agreed(self) -> None:
        """``check`` agreed on by every rank: the channels' error words are MAX-reduced, so
        a timeout seen by one rank raises on ALL ranks together (no rank is left waiting in
        the next collective while another tears down)."""
        if not self.ctx.enabled:
            return
        bad = 0
        if self.xgmi is not None:
            bad = int(any(ch.error() for ch in self.xgmi.channels.values()))
        if any(f() for f in self.extra_errors):
            bad = 1
        flag = torch.tensor([bad], dtype=torch.int32, device=self.ctx.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item():
            raise RuntimeError("peer-buffer transport timed out waiting for a peer on some rank "
                               "(xGMI channel / async_ps state poisoned)")

    def _xg_channel(self, tag: str, srcs, dsts=None) -> Optional["_xg.XgmiChannel"]:
        """The xGMI channel for call site ``tag``, or None for RCCL.  Decided once per tag,
        collectively (same answer on every rank): the messages must fit the kernel's
        alignment rules, and under ``CSA_XGMI=auto`` both paths are timed on scratch
        copies of the real tensors (each as a HIP graph of 10 calls) and the faster wins."""
        if self.xgmi is None:
            return None
        if tag in self._choice:
            return self._choice[tag]
        if torch.cuda.is_current_stream_capturing():
            if self.det:
                raise RuntimeError(f"deterministic collective {tag!r} first used inside graph capture")
            return None                  # undecided inside capture: RCCL (same on all ranks)
        nbytes = sum(t.numel() * t.element_size() for t in srcs)
        try:
            ch = self.xgmi.channel(tag, nbytes)
        except RuntimeError as exc:      # raised on every rank together (collective agreement)
            self.xgmi_tuning[tag] = {"bytes": nbytes, "error": str(exc)}
            self._choice[tag] = None
            return None
        ok = ch.fits(srcs) and (dsts is None or all(d.is_contiguous() and d.data_ptr() % 16 == 0 for d in dsts))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.ctx.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        choice = ch if flag.item() else None
        if choice is not None and self.xgmi_mode == "auto" and not self.det:
            times = self._time_paths(ch, srcs, dsts)
            rc_us = times.pop("rccl")
            proto = min(times, key=times.get)
            xg_us = times[proto]
            self.xgmi_tuning[tag] = {"bytes": nbytes, "rccl_us": round(rc_us, 2),
                                     **{f"{k}_us": round(v, 2) for k, v in times.items()}}
            if dsts is None:
                ch.protocol = proto       # all-reduce: the faster xGMI protocol
                self.xgmi_tuning[tag]["protocol"] = proto
            # a peer wait that timed out during the timing poisons the channel (and would
            # make it look fast): every rank then drops it and stays on RCCL
            healthy = torch.tensor([0 if ch.error() else 1], dtype=torch.int32, device=self.ctx.device)
            dist.all_reduce(healthy, op=dist.ReduceOp.MIN)
            if not healthy.item():
                self.xgmi_tuning[tag]["error"] = "peer wait timed out"
                ch.close()
                del self.xgmi.channels[tag]
                choice = None
            elif not xg_us < rc_us:
                choice = None
        self._choice[tag] = choice
        return choice

    def _time_paths(self, ch, srcs, dsts) -> Dict[str, float]:
        """µs per call of each candidate (max over ranks): all-reduce sites time the
        one-shot and two-shot xGMI protocols and RCCL; gather sites xGMI and RCCL."""
        ss = [torch.zeros_like(t) for t in srcs]
        sd = None if dsts is None else [torch.empty_like(d) for d in dsts]

        def one():
            if sd is None:
                ch.all_reduce(ss, protocol="oneshot")
            else:
                ch.all_gather(list(zip(ss, sd)))

        def two():
            ch.all_reduce(ss, protocol="twoshot")

        def rc():
            for i, t in enumerate(ss):
                if sd is None:
                    dist.all_reduce(t, group=self._pg())
                else:
                    dist.all_gather_into_tensor(sd[i], t, group=self._pg())

        cands = {"oneshot" if sd is None else "xgmi": one, "rccl": rc}
        if sd is None and self.ctx.world > 2:
            cands["twoshot"] = two
        return self._time_fns(cands)

    def _tune_side(self):
        """The tuner's warm-up stream (outside torch's stream pool: utils/streams.py)."""
        if getattr(self, "_tside", None) is None:
            from ..utils.streams import dedicated_stream
            self._tside = dedicated_stream(self.ctx.device)
        return self._tside

    def _time_fns(self, cands) -> Dict[str, float]:
        """µs per call of each candidate callable (max over ranks): an eager warm-up (RCCL
        communicator paths), then a HIP graph of 10 calls replayed 3 times."""
        dev = self.ctx.device
        out = []
        for fn in cands.values():
            side = self._tune_side()
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                fn()                          # eager warm-up (RCCL communicator paths)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with capture(g):
                for _ in range(10):
                    fn()
            g.replay()
            torch.cuda.synchronize(dev)
            dist.all_reduce(torch.zeros(1, device=dev))   # line the ranks up
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                g.replay()
            b.record()
            torch.cuda.synchronize(dev)
            out.append(a.elapsed_time(b) * 1e3 / 30)
            del g
        t = torch.tensor(out, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return {k: float(v) for k, v in zip(cands, t.tolist())}

    @property
    def grad_scale(self) -> float:
        """Factor folded into dL/dlogits so that SUM-reduced grads are the global mean."""
        if self.strategy == "async_ps":
            return 1.0        # each push is ONE worker's update, applied on its own (PS semantics)
        return 1.0 / self.ctx.world if self.ctx.enabled else 1.0

    def shard_range(self) -> Tuple[int, int]:
        if not self.sharded:
            return 0, self.numel
        r = self.ctx.rank
        return r * self.shard, (r + 1) * self.shard

    def buckets(self, lo: int = 0, hi: Optional[int] = None) -> List[Tuple[int, int]]:
        hi = self.numel if hi is None else hi
        out, o = [], lo
        while o < hi:
            out.append((o, min(hi, o + self.bucket_elems)))
            o = out[-1][1]
        return out

    # ---- allreduce ----
    def allreduce(self, flat_grad: torch.Tensor, lo: int = 0, hi: Optional[int] = None) -> None:
        if not self.ctx.enabled:
            return
        for a, b in self.buckets(lo, hi):
            ch = self._xg_channel(f"ar:{a}:{b}", [flat_grad[a:b]])
            with self._timed():
                if ch is not None:
                    ch.all_reduce([flat_grad[a:b]])
                elif self.det:
                    self._det_sum(flat_grad[a:b])
                else:
                    dist.all_reduce(flat_grad[a:b], group=self._pg())

    # ---- deterministic fallback (no xGMI channel) ----
    def _det_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape]: every rank's copy of ``t`` (exact: an all-gather moves bits)."""
        out = torch.empty((self.ctx.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1), group=self._pg())
        return out

    def _det_sum(self, t: torch.Tensor) -> None:
        """In-place SUM over ranks, added in rank order 0, 1, .. W-1 on every rank."""
        g = self._det_gather(t)
        acc = g[0].clone()
        for r in range(1, self.ctx.world):
            acc.add_(g[r])
        t.copy_(acc)

    # ---- ps (sharded) ----
    def reduce_scatter(self, flat_grad: torch.Tensor, shard_out: torch.Tensor) -> None:
        if not self.ctx.enabled:
            shard_out.copy_(flat_grad)
            return
        if self.det or self.xgmi is not None:
            # one range covering the buffer: the xGMI range kernel where it was measured
            # faster (or deterministic mode), else RCCL's reduce-scatter
            self.reduce_scatter_range(flat_grad, shard_out, 0, self.numel)
            return
        with self._timed():
            dist.reduce_scatter_tensor(shard_out, flat_grad, group=self._pg())

    def rs_choice(self, flat_grad: torch.Tensor, shard_out: torch.Tensor, lo: int, hi: int):
        """The path of the [lo, hi) range reduce-scatter, decided once per range and
        collectively: the xGMI range kernel if the range fits its alignment rules and —
        under ``CSA_XGMI=auto`` — it measured faster than RCCL on scratch copies (each as
        a HIP graph of 10 calls, recorded under ``xgmi_tuning['rs:lo:hi']``); else None
        (RCCL).  ``CSA_XGMI=1`` and deterministic mode take xGMI whenever it fits."""
        tag = f"rs:{lo}:{hi}"
        if tag in self._choice:
            return self._choice[tag]
        if self.xgmi is None:
            return None
        if torch.cuda.is_current_stream_capturing():
            if self.det:
                raise RuntimeError(f"deterministic collective {tag!r} first used inside graph capture")
            return None
        sh = self.shard
        ok = lo % 4 == 0 and hi % 4 == 0 and sh % 4 == 0 and flat_grad.data_ptr() % 16 == 0 \
            and shard_out.data_ptr() % 16 == 0
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.ctx.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ch = self.xgmi.channel(tag, (hi - lo) * 4) if flag.item() else None
        if ch is not None and self.xgmi_mode == "auto" and not self.det:
            sf, so = torch.zeros_like(flat_grad), torch.zeros_like(shard_out)
            times = self._time_fns({"xgmi": lambda: ch.reduce_scatter_range(sf, lo, hi, sh, so),
                                    "rccl": lambda: self._rs_rccl(sf, so, lo, hi)})
            self.xgmi_tuning[tag] = {"bytes": (hi - lo) * 4, "xgmi_us": round(times["xgmi"], 2),
                                     "rccl_us": round(times["rccl"], 2)}
            healthy = torch.tensor([0 if ch.error() else 1], dtype=torch.int32, device=self.ctx.device)
            dist.all_reduce(healthy, op=dist.ReduceOp.MIN)
            if not healthy.item():
                self.xgmi_tuning[tag]["error"] = "peer wait timed out"
                ch.close()
                del self.xgmi.channels[tag]
                ch = None
            elif not times["xgmi"] < times["rccl"]:
                ch = None
        self._choice[tag] = ch
        return ch

    def _rs_rccl(self, flat_grad: torch.Tensor, shard_out: torch.Tensor, lo: int, hi: int) -> None:
        """RCCL form of the range reduce-scatter: the whole buffer is one reduce-scatter,
        a partial range one reduce per owner portion."""
        sh, W, r = self.shard, self.ctx.world, self.ctx.rank
        if lo == 0 and hi == self.numel and self.ctx.backend != "gloo":
            dist.reduce_scatter_tensor(shard_out, flat_grad, group=self._pg())
            return
        for p in range(W):
            a, b = max(lo, p * sh), min(hi, (p + 1) * sh)
            if a >= b:
                continue
            part = flat_grad[a:b]
            if self.ctx.backend == "gloo":
                buf = part.clone()
                dist.reduce(buf, dst=p, group=self._pg())
                if p == r:
                    shard_out[a - r * sh:b - r * sh].copy_(buf)
            else:
                dist.reduce(part, dst=p, group=self._pg())
                if p == r:
                    shard_out[a - r * sh:b - r * sh].copy_(part)

    def reduce_scatter_range(self, flat_grad: torch.Tensor, shard_out: torch.Tensor, lo: int, hi: int) -> None:
        """The [lo, hi) part of ``reduce_scatter``: every element is summed into its owner's
        shard (owner = index // shard).  Issued per gradient bucket as the backward produces
        it (the HIP program's overlapped ps step); once every bucket covering the buffer has
        run, ``shard_out`` equals ``reduce_scatter``'s.  xGMI (where ``rs_choice`` picked
        it): one launch, each element leaves its GPU at most once; otherwise RCCL."""
        if not self.ctx.enabled:
            shard_out[lo:hi].copy_(flat_grad[lo:hi])
            return
        sh, r = self.shard, self.ctx.rank
        ch = self.rs_choice(flat_grad, shard_out, lo, hi)
        with self._timed():
            if ch is not None:
                ch.reduce_scatter_range(flat_grad, lo, hi, sh, shard_out)
                return
            if self.det:
                a, b = max(lo, r * sh), min(hi, (r + 1) * sh)
                part = flat_grad[lo:hi].clone()
                self._det_sum(part)              # (every rank sums the range; keeps its part)
                if a < b:
                    shard_out[a - r * sh:b - r * sh].copy_(part[a - lo:b - lo])
                return
            self._rs_rccl(flat_grad, shard_out, lo, hi)

    def all_gather_params(self, flat_param: torch.Tensor) -> None:
        """Every owner's updated shard to every rank (xGMI: one push of the shard to the 7
        peers at once; else RCCL all-gather)."""
        if not self.ctx.enabled:
            return
        lo, hi = self.shard_range()
        ch = None
        if self.ctx.backend == "nccl":
            ch = self._xg_channel("ps_ag", [flat_param[lo:hi]], [flat_param])
        with self._timed():
            if ch is not None:
                ch.all_gather([(flat_param[lo:hi], flat_param)])
                return
            dist.all_gather_into_tensor(flat_param, flat_param[lo:hi].clone()
                                        if self.ctx.backend == "gloo" else flat_param[lo:hi], group=self._pg())

    # ---- lowrank ----
    def all_gather_rows(self, local: torch.Tensor, out: torch.Tensor) -> None:
        """[B, n] per rank -> [world*B, n] (rank-major)."""
        if not self.ctx.enabled:
            out.copy_(local)
            return
        dist.all_gather_into_tensor(out, local.contiguous(), group=self._pg())

    def all_gather_rows_many(self, pairs, tag: str = "gather") -> None:
        """Several ``all_gather_rows`` issued as ONE launch where the xGMI peer-buffer kernel
        takes them (each separate RCCL collective pays its own fixed latency).  ``tag`` names the call site (one
        device-ordered sequence of calls per tag)."""
        if not self.ctx.enabled:
            for local, out in pairs:
                out.copy_(local)
            return
        ch = self._xg_channel(tag, [p[0] for p in pairs], [p[1] for p in pairs]) if len(pairs) <= 8 else None
        with self._timed():
            if ch is not None:
                ch.all_gather(pairs)
                return
            for local, out in pairs:
                dist.all_gather_into_tensor(out, local.contiguous(), group=self._pg())

    def allreduce_ranges(self, flat: torch.Tensor, ranges, tag: str = "ranges") -> None:
        """Sum-all-reduce the given [lo, hi) slices of ``flat`` (one launch on the xGMI
        kernel, else one RCCL all-reduce per slice)."""
        if not self.ctx.enabled or not ranges:
            return
        ch = self._xg_channel(tag, [flat[lo:hi] for lo, hi in ranges]) if len(ranges) <= 8 else None
        with self._timed():
            if ch is not None:
                ch.all_reduce([flat[lo:hi] for lo, hi in ranges])
                return
            for lo, hi in ranges:
                if self.det:
                    self._det_sum(flat[lo:hi])
                else:
                    dist.all_reduce(flat[lo:hi], group=self._pg())

    def allreduce_tensors(self, tensors, tag: str) -> None:
        """In-place SUM of small fp32 tensors across ranks (SyncBN statistics slabs)."""
        if not self.ctx.enabled:
            return
        ch = self._xg_channel(tag, list(tensors)) if len(tensors) <= 8 else None
        with self._timed():
            if ch is not None:
                ch.all_reduce(list(tensors))
                return
            for t in tensors:
                if self.det:
                    self._det_sum(t)
                else:
                    dist.all_reduce(t, group=self._pg())

    def broadcast_params(self, flat_param: torch.Tensor) -> None:
        """Initial sync from rank 0 (reference: chief runs init_op, construct_distribute.py:379)."""
        if self.ctx.enabled:
            dist.broadcast(flat_param, src=0)

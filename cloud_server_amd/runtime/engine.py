"""Training engine: one step = gather batch -> fwd -> bwd -> grad sync -> optimizer.

Replaces the reference worker loop (construct_distribute.py:385-421), where every
``sess.run(train_op)`` pulled all variables from the PS over gRPC, ran fwd/bwd on one
CPU and pushed gradients back (≈142 ms per B=50 step, API.md:462-507).

MI355X design:
* the dataset is resident in HBM and batches are gathered on device (``BatchStream``),
* the whole step — gather, forward, backward, gradient all-reduce, optimizer and the
  accuracy/loss bookkeeping — is captured ONCE into a HIP graph and replayed, so a step
  costs one ``hipGraphLaunch`` and zero host syncs,
* two step programs share that contract:
  - ``TorchProgram``: autograd over eager PyTorch ops (CPU path, reference numerics),
  - ``HipProgram`` (``runtime.hip_program``): the hand-written CDNA4 kernels
    (``ops.fused``) with an explicit backward and the fused optimizer,
* metrics (per-step correct count and loss) go to a device ring buffer that the host
  reads only every ``log_every`` steps (the reference logs every 100, :405).
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import torch

from ..data.datasets import ArrayDataset
from ..data.stream import BatchStream, DeviceDataset
from ..models.cnn import DigitNet, build_model, loss_fn
from ..models.dsl import TrainConfig
from ..ops import optim_ref
from ..parallel.dist import DistContext, ranks_share_gpu
from ..parallel.dp import GradSync
from ..utils.tracing import trace_range
from ..utils.graphs import capture

RING = 4096


def deterministic_mode() -> bool:
    import os
    return os.environ.get("CSA_DETERMINISTIC", "0") == "1"


def enable_deterministic_torch() -> None:
    import os
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


class StepProgram:
    """Interface: ``run()`` performs one full training step on device (capturable)."""

    def run(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class TorchProgram(StepProgram):
    def __init__(self, eng: "TrainEngine"):
        self.e = eng

    def run(self) -> None:
        e = self.e
        idx = e.stream.current()
        x, y = e.data.batch(idx)
        logits = e.model(x)
        loss = loss_fn(e.cfg.loss_name, logits, y)
        e.flat_grad.zero_()
        (loss * e.sync.grad_scale).backward()
        with torch.no_grad():
            e.apply_update()
            correct = (logits.argmax(1) == y).sum().to(torch.int32)
            e.record(correct, loss.detach())


class TrainEngine:
    def __init__(self, cfg: TrainConfig, train: ArrayDataset, device="cpu",
                 ctx: Optional[DistContext] = None, backend: str = "auto",
                 use_graph: Optional[bool] = None, strategy: str = "allreduce",
                 stream_chunk: int = 512, packed: bool = False):
        """``packed``: this engine will run as one branch of a multi-job graph
        (``runtime.multijob``): its HIP program uses the packed launch profile."""
        self.cfg = cfg
        self.packed = packed
        # "<strategy>:hf" — the data-parallel program with the one-GPU step's structure
        # (dense weight gradients formed inside the pair backward launch, no bucket overlap);
        # the start-up tuner times it against the overlapped program (parallel/strategy.py)
        strategy, _, variant = strategy.partition(":")
        if strategy == "async_ps" and not variant:
            # async_ps runs the ":hf" program by default (world 1: 0.0997 against 0.1112
            # ms/step for the bucketed one, profiles/r6_notes.md); "async_ps:flat" (or
            # CSA_APS_VARIANT=flat) keeps the bucketed program
            variant = os.environ.get("CSA_APS_VARIANT", "hf")
        self.dp_variant = "" if variant == "flat" else variant
        if deterministic_mode() and strategy == "lowrank" and ctx is not None and ctx.enabled:
            # same exact DP math; its gathered-operand GEMMs have no fixed-order variant
            strategy = "allreduce"
        self.ctx = ctx or DistContext(device=torch.device(device))
        self.device = torch.device(device)
        # CSA_SHARED_GPU_PROFILE=0 keeps the one-rank-per-GPU launch shapes even when ranks
        # share a device (reproduces the round-5 world-2 stall: scripts/xgmi_stress.py)
        self.shared_gpu = (ranks_share_gpu(self.ctx, self.device)
                           and os.environ.get("CSA_SHARED_GPU_PROFILE", "1") != "0")
        self.model: DigitNet = build_model(cfg, self.device, pad_multiple=self.ctx.world,
                                           dense_last=strategy == "lowrank")
        self.model.train()
        self.model.sync_bn = bool(cfg.sync_bn and self.ctx.enabled)
        self.flat = self.model.flat.data
        self.flat_grad = torch.zeros_like(self.flat)
        self.model.flat.grad = self.flat_grad
        self.sync = GradSync(self.ctx, self.flat.numel(), strategy)
        self.sync.broadcast_params(self.flat)
        self.opt_id = optim_ref.OPT_IDS[cfg.effective_optimizer]
        self.lr = cfg.effective_lr
        lo, hi = self.sync.shard_range()
        self.slots = optim_ref.init_slots(self.opt_id, hi - lo, self.device)
        self.grad_shard = torch.zeros(hi - lo, device=self.device) if strategy == "ps" else None
        # asynchronous bounded-staleness PS (parallel/async_ps.py): the reference's own
        # semantics — pushes applied one by one by their shard's owner as they arrive
        self.aps = None
        if strategy == "async_ps" and self.ctx.enabled:
            from ..parallel.async_ps import make_async_ps
            self.aps = make_async_ps(self, lo, hi)
            if hasattr(self.aps, "error"):
                # a timed-out peer wait freezes the device transport (every later launch
                # returns at once): part of the ranks' agreed health check
                self.sync.extra_errors.append(self.aps.error)
        self.data = DeviceDataset(train, self.device)
        self.stream = BatchStream(self.data.n, cfg.batch_size, self.device, seed=cfg.seed,
                                  chunk=stream_chunk, rank=self.ctx.rank, world=self.ctx.world)
        # device-side counters / metric rings (read by host every log interval)
        self.dstep = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.ring_correct = torch.zeros(RING, dtype=torch.int32, device=self.device)
        self.ring_loss = torch.zeros(RING, dtype=torch.float32, device=self.device)
        self.host_step = 0
        # CSA_DETERMINISTIC=1: bitwise-reproducible steps for tests and
        # debugging.  The HIP program keeps its kernels and swaps every cross-workgroup
        # float atomic for exclusive rows + fixed-order folds (det.hip); a network outside
        # that family runs on the eager program with PyTorch's deterministic algorithms and
        # atomics-free pooling.  Either way still captured in a HIP graph
        self.deterministic = deterministic_mode()
        if backend == "auto":
            backend = "hip" if self.device.type == "cuda" else "torch"
        self.backend = backend
        self.fallback_reason = ""
        if backend == "hip":
            from .hip_program import HipProgram, Unsupported
            try:
                self.program: StepProgram = HipProgram(self)
            except Unsupported as exc:   # config outside the fused-kernel family
                self.fallback_reason = str(exc)
                self.backend = backend = "torch"
        if backend == "torch":
            if self.deterministic:
                # the eager program: PyTorch's deterministic algorithms + gather-form pooling
                enable_deterministic_torch()
                self.model.deterministic = True
            self.program = TorchProgram(self)
        # an in-kernel bounded wait that timed out (the pair backward's tail) is part of the
        # ranks' agreed health check under data parallelism, like a poisoned xGMI channel
        if hasattr(self.program, "health_words"):
            self.sync.extra_errors.append(lambda: any(int(w.item()) for w in self.program.health_words()))
        # the program re-stages its batch whenever the host moves the cursor (seek/resume)
        self.stream.on_reset = (lambda: self.program.prime()) if hasattr(self.program, "prime") else None
        if use_graph is None:
            use_graph = self.device.type == "cuda"
        self.use_graph = use_graph and self.device.type == "cuda"
        self.graph = None
        self.graph_k = None      # CSA_GRAPH_STEPS steps captured in one graph (run_steps)
        # further multi-step graph sizes to capture beside k, k/2, .. (a known loop length:
        # bench.py's K timed steps replay as ONE graph, no inter-graph gaps)
        self.extra_group_sizes: List[int] = []
        self.graphs_k: Dict[int, object] = {}   # every multi-step size (group_sizes)
        self.warmed = False      # _warm_up ran (a packed host re-captures without it)

    # ---------------- pieces used by the programs (device ops only) ----------------
    def adam_lr_tensor(self) -> torch.Tensor:
        t = (self.dstep + 1).to(torch.float32)
        return self.lr * torch.sqrt(1 - optim_ref.ADAM_B2 ** t) / (1 - optim_ref.ADAM_B1 ** t)

    def apply_update(self) -> None:
        """Grad sync + optimizer on the flat buffers (torch ops; the HIP program fuses this)."""
        if self.aps is not None:
            self.aps.step(self.flat_grad, self.flat, self.slots)
            return
        if self.sync.strategy == "ps" and self.ctx.enabled:
            lo, hi = self.sync.shard_range()
            self.sync.reduce_scatter(self.flat_grad, self.grad_shard)
            self._opt(self.flat[lo:hi], self.grad_shard, self.slots)
            self.sync.all_gather_params(self.flat)
        else:
            self.sync.allreduce(self.flat_grad)
            self._opt(self.flat, self.flat_grad, self.slots)

    def after_backward_sync(self) -> None:
        """Gradient sync between backward and the (fused) optimizer of the HIP program."""
        if not self.ctx.enabled:
            return
        if self.sync.strategy == "ps":
            self.sync.reduce_scatter(self.flat_grad, self.grad_shard)
        else:
            self.sync.allreduce(self.flat_grad)

    def _opt(self, w, g, slots) -> None:
        if self.opt_id == optim_ref.OPT_ADAM:
            m, v = slots[0], slots[1]
            m.mul_(optim_ref.ADAM_B1).add_(g, alpha=1 - optim_ref.ADAM_B1)
            v.mul_(optim_ref.ADAM_B2).addcmul_(g, g, value=1 - optim_ref.ADAM_B2)
            w.sub_(self.adam_lr_tensor() * m / (v.sqrt() + optim_ref.ADAM_EPS))
        else:
            optim_ref.step_ref(self.opt_id, w, g, slots, self.lr, 1)

    def record(self, correct: torch.Tensor, loss: torch.Tensor) -> None:
        pos = torch.remainder(self.dstep, RING)
        self.ring_correct.index_copy_(0, pos, correct.view(1).to(torch.int32))
        self.ring_loss.index_copy_(0, pos, loss.view(1).to(torch.float32))
        self.dstep.add_(1)

    # ---------------- host API ----------------
    def _warm_up(self, device_sync: bool = True) -> None:
        """Run the program twice off-graph (allocator, autotuning, RCCL comms), then undo
        the warm-up's effect on the model state so capture starts from step 0's state.
        ``device_sync=False``: wait for this engine's streams only (a packed host builds a
        job on a builder thread while the hosted jobs keep stepping)."""
        s = torch.cuda.Stream(self.device)
        snap = self._snapshot()     # parameters, slots, counters, BN running statistics
        s.wait_stream(torch.cuda.current_stream(self.device))     # (after the clones)
        with torch.cuda.stream(s):
            for _ in range(2):      # warm up allocator / autotuning / RCCL comms off-graph
                self.program.run()
            self._join_branch()
        torch.cuda.current_stream(self.device).wait_stream(s)
        if device_sync:
            torch.cuda.synchronize(self.device)
        else:
            s.synchronize()
        # undo the warm-up's effect on the model state
        self._restore(snap)
        self.warmed = True

    def _join_branch(self) -> None:
        """Join the program's pending side-stream branch (HipProgram.join_branch) into the
        current stream: before a capture starts (a capture may not wait on work issued
        outside it) and at the end of every captured sequence (every fork joined)."""
        prog = getattr(self, "program", None)
        if prog is not None and hasattr(prog, "join_branch"):
            prog.join_branch()

    def _capture(self) -> None:
        self._warm_up()
        g = torch.cuda.CUDAGraph()
        self._join_branch()
        # thread_local: the RCCL watchdog thread queries events of earlier collectives while
        # this thread captures; in "global" mode that query aborts the process
        with capture(g):
            self.program.run()
            self._join_branch()
        self.graph = g
        # capture does not execute: the cursor/step still point at this step

    def step(self) -> None:
        self.stream.before_step()
        with trace_range("csa.step"):          # ROCTx range when CSA_TRACE=1
            if self.use_graph:
                if self.graph is None:
                    with trace_range("csa.capture"):
                        self._capture()
                self.graph.replay()
            else:
                self.program.run()
        self.host_step += 1

    def group_steps(self) -> int:
        """Steps per multi-step graph (1: grouping off — eager, or CSA_GRAPH_STEPS=1).
        Under data parallelism every collective of a step is already captured in the
        single-step graph (RCCL kernels, or the xGMI peer-buffer kernels whose channel
        sequence numbers live on the device), so k steps capture the same way; the
        per-call-site path choice is made eagerly at warm-up, before any capture."""
        k = int(os.environ.get("CSA_GRAPH_STEPS", "32"))
        if self.ctx.enabled and os.environ.get("CSA_DP_GRAPH_STEPS", "1") != "1":
            return 1
        return k if (self.use_graph and k > 1) else 1

    def group_sizes(self) -> List[int]:
        """Multi-step graph sizes, largest first: k, k/2, ..., 2 (k = ``group_steps``), so
        any ``n`` decomposes into at most one replay per size plus whole k-groups."""
        k = self.group_steps()
        sizes = []
        while k > 1:
            sizes.append(k)
            k //= 2
        if self.group_steps() > 1:
            sizes = sorted(set(sizes) | {n for n in self.extra_group_sizes if n > 1}, reverse=True)
        return sizes

    def _snapshot(self):
        """Model / optimizer / stream state a throw-away replay must not change."""
        return ((self.flat.clone(), self.slots.clone(), self.dstep.clone(), self.stream.cursor.clone()),
                [(b, b.clone()) for b in self.model.buffers()])

    def _restore(self, snap) -> None:
        (flat, slots, dstep, cursor), bufs = snap
        self.flat.copy_(flat); self.slots.copy_(slots)
        self.dstep.copy_(dstep); self.stream.cursor.copy_(cursor)
        for b, v in bufs:
            b.copy_(v)
        if self.aps is not None and hasattr(self.aps, "reset"):
            self.aps.reset()             # async_ps mailboxes / clocks back to step 0 (collective)
        if hasattr(self.program, "reset_after_warmup"):
            self.program.reset_after_warmup()

    def prepare_group_graph(self) -> None:
        """Capture every multi-step graph now (``group_sizes``: k, k/2, .., 2 steps each) and
        replay each ONCE with the model state restored afterwards, so neither a capture nor
        a graph's first launch (its upload to the device) ever lands in a timed loop.  Call
        after the first step (the single-step graph is then captured and replayed)."""
        if self.graph is None or self.graph_k is not None:
            return
        graphs = {}
        self._join_branch()
        for k in self.group_sizes():
            g = torch.cuda.CUDAGraph()
            with capture(g):
                for _ in range(k):
                    self.program.run()
                self._join_branch()
            graphs[k] = g
        if not graphs:
            return
        self.graphs_k = graphs
        self.graph_k = graphs[max(graphs)]
        # warm replay: the device must not be reading the row table's halves the host
        # refills meanwhile, so drain first; every rank replays the same graphs (collectives
        # inside them stay matched)
        self.sync_device()
        snap = self._snapshot()
        for k in sorted(graphs, reverse=True):
            graphs[k].replay()
        # keep the device busy for ~warm_ms more (throw-away replays of the largest graph:
        # the clocks ramp to their sustained state before any timed loop; measured on
        # MI355X a 20-step loop after a bare warm-up ran 7 % slower than a 2000-step one)
        k = max(graphs)
        warm_ms = float(os.environ.get("CSA_WARM_MS", "100"))
        if self.device.type == "cuda" and warm_ms > 0:
            if self.ctx.enabled:
                # collectives inside: every rank must replay the same count
                for _ in range(16):
                    graphs[k].replay()
            else:
                t0 = time.perf_counter()
                while (time.perf_counter() - t0) * 1e3 < warm_ms:
                    for _ in range(16):
                        graphs[k].replay()
                    self.sync_device()
        self.sync_device()
        self._restore(snap)
        self.sync_device()

    def run_steps(self, n: int) -> None:
        """``n`` training steps.  With a captured single-GPU program, groups of
        ``CSA_GRAPH_STEPS`` (default 32) steps replay ONE graph holding that many steps:
        one launch instead of k.  Bench on MI355X (scripts/gpu_sweep.sh): 0.108 ms/step
        ungrouped, 0.1045 at k = 4, 0.1035 at k = 8, 0.1034 at k = 16; round 5 (scripts/
        gpu_r5x.sh, 2000 steps): 0.08293 at k = 8, 0.08261 at 16, 0.08234 at 32.  The remainder
        ``n mod k`` replays the k/2, k/4, .. 2-step graphs, so at most one step runs as a
        single-step replay.  Groups never straddle a half of the batch row table
        (BatchStream.can_group); exactly ``n`` steps execute."""
        sizes = self.group_sizes() if self.graph is not None else []
        while n > 0:
            k = next((s for s in sizes if s <= n and self.stream.can_group(s)), 1)
            if k > 1:
                self.prepare_group_graph()
                with trace_range("csa.steps"):
                    for _ in range(k):
                        self.stream.before_step()
                    self.graphs_k[k].replay()
                self.host_step += k
                n -= k
            else:
                self.step()
                n -= 1

    def probe_comm(self) -> float:
        """Run THIS step eagerly with every collective bracketed by timing events and
        return its communication time (ms; sum over call sites, side streams included).
        A real training step, so the run's semantics do not change; data parallel only.
        The per-rank value is what ``metrics.jsonl`` reports as ``comm_ms``."""
        if not self.ctx.enabled:
            self.step()
            return 0.0
        if self.use_graph and self.graph is None:
            self._capture()
        self.stream.before_step()
        self.sync.timing = []
        try:
            self.program.run()
        finally:
            ev, self.sync.timing = self.sync.timing, None
        self.host_step += 1
        self.sync_device()
        self._comm_ms = float(sum(a.elapsed_time(b) for a, b in ev))
        return self._comm_ms

    def finish_async(self) -> None:
        """async_ps: apply every outstanding push and pull the final shards (replicas then
        agree); a no-op for the synchronous strategies."""
        if self.aps is not None:
            self.sync_device()
            self.aps.finish(self.flat, self.slots)
            self.sync_device()
            # a timeout anywhere raises on EVERY rank together (never one rank alone)
            self.sync.check_agreed()

    def health_words(self) -> List[torch.Tensor]:
        """Device words that turn nonzero when an in-kernel bounded wait timed out (the
        program's tail); copied without a host sync by the job loop's metric drain."""
        f = getattr(self.program, "health_words", None)
        return list(f()) if f is not None else []

    def check_health(self) -> None:
        """Raise if any in-kernel bounded wait or peer transport timed out: the state is then
        not a valid training state (skipped updates / un-reduced gradients).  Under data
        parallelism the verdict is agreed by every rank (``GradSync.check_agreed``, which
        also reads the program's words); on one rank the words are read here.  A host sync."""
        if self.ctx.enabled:
            self.sync.check_agreed()
            return
        self.sync.check()
        if any(int(w.item()) for w in self.health_words()):
            raise RuntimeError("in-kernel wait timed out (pair-backward tail): conv / BatchNorm "
                               "updates, statistic zeroing or batch staging were skipped")

    def close(self) -> None:
        """Release the peer-buffer transports (collective under data parallelism: every rank
        calls it; buffers go back to the process pool once every rank's kernels drained)."""
        if self.aps is not None and hasattr(self.aps, "close"):
            self.aps.close()
        if self.sync.xgmi is not None:
            self.sync.xgmi.close()

    def staleness(self) -> int:
        """async_ps: the largest parameter staleness (clocks) any step of this rank saw."""
        return int(self.aps.max_staleness) if self.aps is not None else 0

    def comm_ms_per_step(self) -> float:
        return getattr(self, "_comm_ms", 0.0)

    def flush_params(self) -> None:
        """Land a deferred parameter update now, ordered on the current stream (no host
        sync): the data-parallel all-reduce programs apply the dense layers' update in the
        next step's first launch (HipProgram._plan_carry).  Every read of the parameters
        between steps goes through here or through ``sync_device``."""
        prog = getattr(self, "program", None)
        if prog is not None and getattr(prog, "carry", None) is not None:
            prog.flush()

    def sync_device(self) -> None:
        if self.device.type == "cuda":
            self.flush_params()
            torch.cuda.synchronize(self.device)

    def metrics_since(self, start_step: int) -> Dict[str, float]:
        """Mean accuracy/loss of steps [start_step, host_step) (host sync happens here)."""
        n = self.host_step - start_step
        if n <= 0:
            return {"accuracy": float("nan"), "loss": float("nan"), "steps": 0}
        n = min(n, RING)
        pos = [(self.host_step - 1 - i) % RING for i in range(n)]
        idx = torch.tensor(pos, device=self.device)
        c = self.ring_correct.index_select(0, idx).double().sum().item()
        l = self.ring_loss.index_select(0, idx).double().mean().item()
        return {"accuracy": c / (n * self.cfg.batch_size), "loss": l, "steps": n}

    def last_batch_accuracy(self) -> float:
        pos = (self.host_step - 1) % RING
        return float(self.ring_correct[pos].item()) / self.cfg.batch_size

    @torch.no_grad()
    def evaluate(self, ds: ArrayDataset, batch: int = 4096) -> float:
        """Test accuracy with eval-mode BN (running stats unless bn_mode == 'batch')."""
        if len(ds) == 0:
            return float("nan")
        self.model.eval()
        correct = 0
        imgs = torch.from_numpy(ds.images).to(self.device)
        labs = torch.from_numpy(ds.labels).to(self.device)
        for i in range(0, len(ds), batch):
            x = imgs[i:i + batch].float().div_(255.0)
            pred = self.predict_logits(x).argmax(1)
            correct += int((pred == labs[i:i + batch]).sum().item())
        self.model.train()
        return correct / len(ds)

    def predict_logits(self, x: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip" and hasattr(self.program, "predict_logits"):
            return self.program.predict_logits(x)
        return self.model(x)

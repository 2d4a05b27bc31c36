"""Multi-tenant packing: K independent training jobs sharing one MI355X.

The reference ran exactly one job cluster-wide and killed the previous one on every
submit (apps/construction/views.py:128-129); SURVEY §2.3 names packing as the real
throughput lever, because one B=50 step of the sample CNN occupies only part of the 256
CUs for ~126 µs and is bound by kernel latency, not by HBM or MFMA throughput.

Two ways of sharing the card are provided (both measured by ``bench.py --jobs K``):

* ``PackedJobs`` (in-process): each job keeps its own engine (weights, optimizer slots,
  HBM-resident data, batch stream, metric ring), and ONE HIP graph holds a step of every
  job as K independent branches forked onto K streams.  A replay is one
  ``hipGraphLaunch`` and the branches' kernels overlap on the CUs, so the per-kernel
  latency of one job hides behind the work of the others.
* K processes (``runtime.jobs`` slot scheduler): each job is its own process with its own
  HIP context and graph; the hardware queues interleave their launches.

Every job's numerics are exactly those of a lone run: branches share no buffers, and each
branch is the same kernel sequence its own engine would capture.

Packed, the chip is saturated, so what matters is CU-time per job-step rather than one
job's latency: engines built with ``packed=True`` run the packed launch profile (two
pooled rows per conv-pair workgroup, 128-column fused dense blocks; profiles/
r2_multitenant.md) — set per program around its own planning and launches, no process
environment is touched.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .engine import TrainEngine
from ..utils.tracing import trace_range
from ..utils.graphs import capture


class PackedJobs:
    def __init__(self, engines: Sequence[TrainEngine]):
        if not engines:
            raise ValueError("no jobs to pack")
        devs = {e.device for e in engines}
        if len(devs) != 1:
            raise ValueError("packed jobs must share one device")
        self.engines: List[TrainEngine] = list(engines)
        self.device = engines[0].device
        self.cuda = self.device.type == "cuda"
        if any(e.ctx.enabled for e in engines):
            raise ValueError("packed jobs are single-GPU jobs (no data-parallel group)")
        self.graph = None
        self.graph_k = None
        self.host_step = 0

    def _capture_group(self, k: int) -> None:
        """k steps of every job as ONE graph: each job's branch runs its k steps back to
        back (the jobs drift within the graph instead of joining after every step)."""
        streams = self._streams
        g = torch.cuda.CUDAGraph()
        with capture(g):
            cap = torch.cuda.current_stream(self.device)
            for e, s in zip(self.engines, streams):
                s.wait_stream(cap)
                with torch.cuda.stream(s):
                    for _ in range(k):
                        e.program.run()
                    e._join_branch()
            for s in streams:
                cap.wait_stream(s)
        self.graph_k = g

    def prepare_group_graph(self, k: int = 0) -> None:
        """Capture the k-step multi-job graph now and replay it once with every job's state
        restored afterwards (see TrainEngine.prepare_group_graph): a timed loop then never
        pays the capture or the graph's first launch."""
        import os
        k = k or int(os.environ.get("CSA_GRAPH_STEPS", "32"))
        if not self.cuda or k <= 1 or self.graph is None or self.graph_k is not None:
            return
        self._capture_group(k)
        self.sync_device()
        snaps = [e._snapshot() for e in self.engines]
        self.graph_k.replay()
        self.sync_device()
        for e, s in zip(self.engines, snaps):
            e._restore(s)
        self.sync_device()

    def run_steps(self, n: int) -> None:
        """``n`` steps of every job: groups of CSA_GRAPH_STEPS steps as one multi-step
        graph where every job's group stays inside one half of its row table (see
        TrainEngine.run_steps), single packed steps otherwise."""
        import os
        k = int(os.environ.get("CSA_GRAPH_STEPS", "32"))
        while n > 0:
            if (self.cuda and k > 1 and n >= k and self.graph is not None
                    and all(e.stream.can_group(k) for e in self.engines)):
                if self.graph_k is None:
                    self._capture_group(k)
                for _ in range(k):
                    for e in self.engines:
                        e.stream.before_step()
                with trace_range("csa.packed_steps"):
                    self.graph_k.replay()
                for e in self.engines:
                    e.host_step += k
                self.host_step += k
                n -= k
            else:
                self.step()
                n -= 1

    def _capture(self) -> None:
        # only engines that never ran warm up (allocator / library init off-graph); a job
        # already hosted keeps its state untouched and is simply captured again, so an
        # admission or retirement costs one graph capture, not 2 eager steps per tenant
        for e in self.engines:
            if not e.warmed:
                e._warm_up()
        main = torch.cuda.current_stream(self.device)
        from ..utils.streams import dedicated_stream
        if len(getattr(self, "_own_streams", [])) < len(self.engines):
            self._own_streams = [dedicated_stream(self.device) for _ in self.engines]
        streams = self._own_streams[:len(self.engines)]
        g = torch.cuda.CUDAGraph()
        with capture(g):
            cap = torch.cuda.current_stream(self.device)
            for e, s in zip(self.engines, streams):
                s.wait_stream(cap)            # fork: each job a branch of the graph
                with torch.cuda.stream(s):
                    e.program.run()
                    e._join_branch()
            for s in streams:
                cap.wait_stream(s)            # join
        self.graph = g
        self._streams = streams
        del main

    def step(self) -> None:
        """One step of every job."""
        for e in self.engines:
            e.stream.before_step()
        with trace_range("csa.packed_step"):
            if self.cuda:
                if self.graph is None:
                    self._capture()
                self.graph.replay()
            else:
                for e in self.engines:
                    e.program.run()
        for e in self.engines:
            e.host_step += 1
        self.host_step += 1

    def sync_device(self) -> None:
        if self.cuda:
            torch.cuda.synchronize(self.device)

    @property
    def samples_per_step(self) -> int:
        return sum(e.cfg.batch_size * e.ctx.world for e in self.engines)

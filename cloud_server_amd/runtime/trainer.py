"""One training job: dataset -> engine -> loop with logging, checkpoints, control.

Reference job body: construct_distribute.py:325-421 (user JPEGs + tag.json) and
construct_distribute_url.py (stock MNIST).  Kept behaviour:

* ``result.txt`` in the model dir, append mode, one ``step:%d,accuracy:%f,duration:%f``
  line every ``log_every`` (100) steps — accuracy is the batch accuracy at that step,
  duration the wall time of the previous train step — then ``final_accuracy:%f`` + a
  blank line (:405-420).  The URL variant's missing final line (quirk 5) is fixed.
* resume from the newest checkpoint in ``train_model/`` (Supervisor auto-restore).

New: ``metrics.jsonl`` (step, loss, accuracy, step_ms, samples_per_s), ``status.json``
(state machine queued -> running -> paused -> stopped | failed | done), a control
file (``control.json``: stop / pause / resume) polled between log intervals, an
optional fault-injection hook (``CSA_FAULT_AT_STEP``) for failure-recovery tests, and
multi-GPU data parallel when launched under ``torch.distributed``.
"""
from __future__ import annotations

import json
import os
import time
import traceback
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..data.datasets import ArrayDataset, load_dataset_for_model, load_mnist_dir
from ..models.dsl import parse_train_config
from ..parallel.dist import DistContext, all_reduce_max, barrier
from . import checkpoint as ckpt
from ..utils.locks import WriterLock
from ..utils.tracing import trace_range
from .engine import TrainEngine

RESULT = "result.txt"
METRICS = "metrics.jsonl"
STATUS = "status.json"
CONTROL = "control.json"


def write_status(model_dir: str, **fields) -> None:
    p = os.path.join(model_dir, STATUS)
    cur: Dict[str, Any] = {}
    if os.path.exists(p):
        try:
            with open(p) as f:
                cur = json.load(f)
        except (OSError, json.JSONDecodeError):
            cur = {}
    cur.update(fields)
    cur["updated"] = time.time()
    tmp = p + ".tmp"
    with open(tmp, "w") as f:
        json.dump(cur, f)
    os.replace(tmp, p)


def read_control(model_dir: str) -> str:
    p = os.path.join(model_dir, CONTROL)
    try:
        with open(p) as f:
            return str(json.load(f).get("action", ""))
    except (OSError, json.JSONDecodeError):
        return ""


def load_job_data(model_dir: str, datatype: str, ratio: float):
    """(train, test) splits.  'url' -> MNIST idx files (train/t10k); 'file' -> JPEGs
    under model_dir/data labelled by model_dir/tag.json, ordered split at int(N*ratio)."""
    data_dir = os.path.join(model_dir, "data")
    if datatype == "url":
        train, test = load_mnist_dir(data_dir)
        if test is None:
            train, test = train.split(ratio)
        return train, test
    ds = load_dataset_for_model(data_dir, os.path.join(model_dir, "tag.json"), "file")
    if len(ds) == 0:
        raise ValueError("no labelled images found (check tag.json and the data folder)")
    train, test = ds.split(ratio)
    if len(train) == 0:
        train = ds
    return train, test


def _fault_step(rank: int, model_dir: str) -> int:
    """``CSA_FAULT_AT_STEP``: ``s`` (every rank raises at step s) or ``k:s`` (only rank k):
    the "kill rank k at step s" hook of SURVEY.md §5.3.  With ``CSA_FAULT_ONCE=1`` the
    fault fires on the first attempt only (a marker file in the model dir), so a test can
    watch the automatic restart succeed."""
    v = os.environ.get("CSA_FAULT_AT_STEP", "").strip()
    if not v:
        return -1
    if os.environ.get("CSA_FAULT_ONCE", "0") == "1":
        marker = os.path.join(model_dir, ".fault_fired")
        if os.path.exists(marker):
            return -1
        open(marker, "w").close()
    if ":" in v:
        r, st = v.split(":", 1)
        return int(st) if int(r) == rank else -1
    return int(v)


def _tail_timeout_step(model_dir: str) -> int:
    """``CSA_TAIL_TIMEOUT_AT_STEP=s``: arm the HIP program's forced tail timeout
    (``HipProgram.arm_tail_timeout``) before step ``s`` — the in-kernel failure a starved
    pair workgroup would cause.  Fires once per model dir (a marker file), so the
    automatic restart from the last checkpoint can be watched to succeed."""
    v = os.environ.get("CSA_TAIL_TIMEOUT_AT_STEP", "").strip()
    if not v:
        return -1
    marker = os.path.join(model_dir, ".tail_timeout_fired")
    if os.path.exists(marker):
        return -1
    open(marker, "w").close()
    return int(v)


def _strip_final_tail(path: str, resume_step: int) -> None:
    """A resumed (extended or restarted) job appends its step lines after the previous
    run's; first drop that run's ``final_accuracy`` tail and every row at or after the step
    it resumes from (a restart from an older checkpoint re-logs them; the compat row at
    step == iter, see ``JobRun.finish``), so the file stays one run of increasing step
    lines and then one final line — the reference monitor reads only up to the first
    non-step line (apps/runtime/views.py:55)."""
    if not os.path.exists(path):
        return
    with open(path) as f:
        lines = f.readlines()
    keep = 0
    while keep < len(lines) and lines[keep].startswith("step"):
        try:
            st = int(lines[keep].split(",")[0].split(":")[1])
        except (IndexError, ValueError):
            break
        if st >= resume_step:
            break
        keep += 1
    if keep < len(lines):
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.writelines(lines[:keep])
        os.replace(tmp, path)


class _MetricLog:
    """Training-log lines without stalling the device queue.

    At a log step the engine's device metric rings are copied into pinned host memory
    (non-blocking, stream-ordered) and a timing event is recorded; the line is written
    once that event has completed — normally at the next log point, so the host never
    waits for the GPU to drain.  Durations come from the device events (mean step time
    over the interval).  CPU runs are synchronous and write immediately."""

    def __init__(self, eng: TrainEngine, chief: bool, result_path: str, metrics_path: str, world: int):
        from collections import deque
        self.eng, self.chief, self.world = eng, chief, world
        self.cuda = eng.device.type == "cuda"
        self.pending = deque()
        self.prev_ev = None
        self.prev_step = None
        self.t_host = time.perf_counter()
        self.h_step = eng.host_step
        self.last_acc = float("nan")
        if chief:
            _strip_final_tail(result_path, eng.host_step)
        self.fr = open(result_path, "a") if chief else None
        self.fm = open(metrics_path, "a") if chief else None
        self.lines = 0
        self.last_dt = 0.0
        # one rank: the in-kernel timeout words ride with the metric copies (no host sync)
        # and a nonzero one fails the job when its log line drains; under data parallelism
        # the ranks' agreed check at control points reads them instead
        self.health = eng.health_words() if world == 1 else []

    def mark(self, step: int, int_start: int) -> None:
        e = self.eng
        if self.cuda:
            pc = torch.empty(e.ring_correct.shape, dtype=e.ring_correct.dtype, pin_memory=True)
            pl = torch.empty(e.ring_loss.shape, dtype=e.ring_loss.dtype, pin_memory=True)
            pc.copy_(e.ring_correct, non_blocking=True)
            pl.copy_(e.ring_loss, non_blocking=True)
            ph = None
            if self.health:
                ph = torch.empty(len(self.health), dtype=torch.int32, pin_memory=True)
                for i, w in enumerate(self.health):
                    ph[i:i + 1].copy_(w, non_blocking=True)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream(e.device))
            self.pending.append((step, int_start, e.host_step, ev, pc, pl, time.perf_counter(), ph))
            self.drain(block=False)
        else:
            self.pending.append((step, int_start, e.host_step, None, e.ring_correct, e.ring_loss,
                                 time.perf_counter(), None))
            self.drain(block=True)

    def drain(self, block: bool) -> None:
        from .engine import RING
        B = self.eng.cfg.batch_size
        while self.pending:
            step, s0, s1, ev, pc, pl, th, ph = self.pending[0]
            if ev is not None and not block and not ev.query():
                return
            self.pending.popleft()
            if ev is not None:
                ev.synchronize()
            if ph is not None and bool(ph.any()):
                raise RuntimeError(f"in-kernel wait timed out by step {s1} (pair-backward tail): "
                                   "parameter updates / statistic zeroing / batch staging skipped")
            n = max(s1 - self.h_step, 1)
            if ev is not None and self.prev_ev is not None:
                step_time = self.prev_ev.elapsed_time(ev) / 1e3 / n
            else:
                step_time = (th - self.t_host) / n
            self.prev_ev, self.t_host, self.h_step = ev, th, s1
            self.last_dt = step_time
            acc = float(pc[step % RING]) / B
            self.last_acc = acc
            k = min(max(s1 - s0, 1), RING)
            pos = [(s1 - 1 - i) % RING for i in range(k)]
            mloss = float(pl[pos].double().mean())
            macc = float(pc[pos].double().sum()) / (k * B)
            if self.chief:
                self.fr.write("step:%d,accuracy:%f,duration:%f\n" % (step, acc, step_time))
                self.fm.write(json.dumps({"step": step, "loss": mloss, "accuracy": macc, "batch_accuracy": acc,
                                          "step_ms": step_time * 1e3,
                                          "samples_per_s": B * self.world / max(step_time, 1e-9),
                                          "comm_ms": self.eng.comm_ms_per_step(),
                                          "time": time.time()}) + "\n")
                self.lines += 1
        if self.chief:
            self.fr.flush()
            self.fm.flush()

    def close(self) -> None:
        self.drain(block=True)
        if self.chief:
            self.fr.close()
            self.fm.close()


class JobRun:
    """One training job's bookkeeping around an engine: resume, logging, heartbeats,
    checkpoints, control actions, fault hooks and the final evaluation.  ``run_job``
    drives it with the job's own engine; ``runtime.gpu_host`` drives several of them
    with one packed graph (``runtime.multijob``), calling ``after_step`` for each job
    after every packed step."""

    def __init__(self, model_dir: str, config: Dict[str, Any], datatype: str = "file",
                 device: Optional[str] = None, ctx: Optional[DistContext] = None,
                 backend: str = "auto", data: Optional[tuple] = None, packed: bool = False):
        self.model_dir = model_dir
        self.ctx = ctx = ctx or DistContext()
        self.chief = chief = ctx.is_chief
        self.cfg = cfg = parse_train_config(config)
        if device is None:
            device = str(ctx.device) if ctx.enabled else ("cuda" if torch.cuda.is_available() else "cpu")
        # single writer per model dir (the reference's shared append-mode result.txt race,
        # SURVEY §5.2): raises LockHeld BEFORE touching status.json of the job that owns it
        self.wlock = WriterLock(model_dir) if chief else None
        if chief:
            write_status(model_dir, state="running", pid=os.getpid(), device=device, world=ctx.world)
        self.ckpter = None
        self.mlog = None
        try:
            train, self.test = data if data is not None else load_job_data(model_dir, datatype, cfg.ratio)
            self.eng = eng = TrainEngine(cfg, train, device=device, ctx=ctx, backend=backend, packed=packed,
                                         strategy=config.get("options", {}).get("strategy", "allreduce")
                                         if isinstance(config.get("options"), dict) else "allreduce")
            if chief:       # which program runs, and why not the HIP one if it does not
                write_status(model_dir, backend=eng.backend, fallback=eng.fallback_reason)
            last = ckpt.latest(model_dir)
            if last is not None:
                ckpt.restore_engine(eng, ckpt.load(last[1]))
            self.fault_at = _fault_step(ctx.rank, model_dir)                       # raise (crash) at this step
            self.tail_timeout_at = _tail_timeout_step(model_dir)                   # forced in-kernel timeout
            self.hang_at = int(os.environ.get("CSA_HANG_AT_STEP", "-1"))   # stop making progress (watchdog tests)
            self.log_every = max(1, cfg.log_every)
            # control / time-checkpoint decisions: every log point on one rank (a file stat); under
            # data parallel they are a broadcast (a sync point), so every ~2000 steps
            self.ctl_every = 1 if not ctx.enabled else max(1, 2000 // self.log_every)
            self.ctl_path = os.path.join(model_dir, CONTROL)
            self.ckpter = ckpt.AsyncCheckpointer(eng, model_dir)
            self.mlog = _MetricLog(eng, chief, os.path.join(model_dir, RESULT),
                                   os.path.join(model_dir, METRICS), ctx.world)
        except Exception as exc:
            self.fail(exc)
            raise
        self.t_ckpt = self.t_status = time.time()
        self.int_start = eng.host_step
        self.nlog = 0
        self.state = "done"

    # ---- the step loop, split so a packed host can interleave several jobs ----
    def pending(self) -> bool:
        return self.eng.host_step < self.cfg.iter

    def before_step(self) -> None:
        """Fault hooks for the step about to run (``eng.host_step``)."""
        step = self.eng.host_step
        if step == self.fault_at:
            raise RuntimeError(f"injected fault at step {step} (rank {self.ctx.rank})")
        if step == self.hang_at:
            while True:
                time.sleep(1.0)
        if step == self.tail_timeout_at:
            arm = getattr(self.eng.program, "arm_tail_timeout", None)
            if arm is None or not arm():
                raise RuntimeError("CSA_TAIL_TIMEOUT_AT_STEP: this program has no pair-backward tail")

    def step(self) -> None:
        eng, ctx = self.eng, self.ctx
        step = eng.host_step
        if ctx.enabled and eng.device.type == "cuda" and step % (self.ctl_every * self.log_every) == 1:
            eng.probe_comm()            # per-rank collective time for metrics.jsonl
            return
        # k steps as one multi-step graph launch (TrainEngine.run_steps) when no per-step
        # hook falls inside them: the group's LAST step may be a log point (after_step
        # handles it), earlier ones may not; fault / hang injection steps run alone
        # (the largest captured size that fits: k, k/2, .., 2 — a log point 4 steps away
        # runs as one 4-step replay instead of four single-step ones)
        sizes = eng.group_sizes() if eng.graph is not None else []
        k = next((s for s in sizes if self.groupable(s)), 1)
        if k > 1:
            eng.run_steps(k)
        else:
            eng.step()

    def groupable(self, k: int) -> bool:
        """May the next ``k`` steps run as one multi-step launch?  Only the group's LAST step
        may be a log point (after_step handles it); fault / hang injection steps run alone."""
        step = self.eng.host_step
        if self.ctx.enabled and self.eng.device.type == "cuda":
            period = self.ctl_every * self.log_every        # comm probe steps run alone
            if any(s % period == 1 for s in range(step, step + k)):
                return False
        return (step + k <= self.cfg.iter
                and all((s % self.log_every) != 0 for s in range(step, step + k - 1))
                and not (step <= self.fault_at < step + k) and not (step <= self.hang_at < step + k)
                and not (step <= self.tail_timeout_at < step + k))

    def after_step(self) -> str:
        """Bookkeeping after step ``host_step - 1`` ran; returns "" to continue, or the
        state that ends the loop ("stopped" / "paused")."""
        eng = self.eng
        step = eng.host_step - 1
        if step % self.log_every != 0:
            return ""
        # reference: the accuracy logged for step s is the batch of step s evaluated
        # with the pre-update weights — exactly this step's forward pass
        with trace_range("csa.log"):
            self.mlog.mark(step, self.int_start)
        self.int_start = eng.host_step
        now = time.time()
        if self.chief and (now - self.t_status > 1.0 or self.nlog == 0):
            write_status(self.model_dir, step=eng.host_step, heartbeat=now)     # watchdog liveness
            self.t_status = now
        self.nlog += 1
        if self.cfg.ckpt_every > 0 and step > 0 and step % self.cfg.ckpt_every == 0:
            eng.check_health()          # never checkpoint a state an in-kernel timeout corrupted
            self.ckpter.save(self.chief)
            self.t_ckpt = now
        if self.nlog % self.ctl_every:
            return ""
        action = ""
        if self.chief:
            action = read_control(self.model_dir) if os.path.exists(self.ctl_path) else ""
            if not action and self.cfg.ckpt_secs > 0 and now - self.t_ckpt >= self.cfg.ckpt_secs:
                action = "ckpt"         # Supervisor(save_model_secs=60), construct_distribute.py:391
        action = _agree(self.ctx, action)
        if self.ctx.enabled:
            # a peer-buffer transport or in-kernel wait that timed out (xGMI channel,
            # async_ps state, the pair-backward tail) stops every rank together, at the
            # next control point, not only at the end
            eng.sync.check_agreed()
        elif action in ("ckpt", "pause"):
            eng.check_health()
        if action == "ckpt":
            with trace_range("csa.ckpt"):
                self.ckpter.save(self.chief)
            self.t_ckpt = now
        elif action == "stop":
            self.state = "stopped"
            return "stopped"
        elif action == "pause":
            self.ckpter.save(self.chief)
            self.ckpter.wait()
            if self.chief:
                write_status(self.model_dir, state="paused", step=eng.host_step)
            self.state = "paused"
            return "paused"
        return ""

    def finish(self) -> Dict[str, Any]:
        eng, state, chief = self.eng, self.state, self.chief
        eng.finish_async()            # async_ps: drain outstanding pushes, pull final shards
        eng.sync_device()
        # a peer wait that timed out after the last log step left this rank's gradient
        # un-reduced, an in-kernel tail wait skipped updates: fail before evaluating /
        # checkpointing diverged parameters (every rank together under data parallelism)
        eng.check_health()
        self.mlog.close()
        final_acc = None
        if state == "done":
            final_acc = eng.evaluate(self.test) if len(self.test) else self.mlog.last_acc
            if chief:
                with open(os.path.join(self.model_dir, RESULT), "a") as f:
                    # the reference's loop (construct_distribute.py:402-414) reads the global
                    # step BEFORE each train op, so it also logs step == iter (and runs one
                    # op more): iter/100 + 1 rows, which is what its monitor's final-line gate
                    # counts on (views.py:66).  This job runs exactly iter steps; its row at
                    # step == iter repeats the final step's batch accuracy
                    if eng.host_step == self.cfg.iter and self.cfg.iter % self.log_every == 0:
                        f.write("step:%d,accuracy:%f,duration:%f\n"
                                % (eng.host_step, eng.last_batch_accuracy(), self.mlog.last_dt))
                    f.write("final_accuracy:%f\n\n" % final_acc)
        if state != "paused":
            self.ckpter.save(chief)
        self.ckpter.wait()
        eng.close()                   # peer buffers back to the pool (collective)
        if chief:
            write_status(self.model_dir, state=state, step=eng.host_step, final_accuracy=final_acc,
                         backend=eng.backend, fallback=eng.fallback_reason)
        self._unlock()
        return {"state": state, "step": eng.host_step, "final_accuracy": final_acc, "backend": eng.backend}

    def fail(self, exc: BaseException) -> None:
        if self.chief:
            step = self.eng.host_step if hasattr(self, "eng") else 0
            write_status(self.model_dir, state="failed", step=step, error=repr(exc),
                         trace=traceback.format_exc()[-4000:])
        try:
            if self.ckpter is not None:
                self.ckpter.wait()      # never leave a half-written checkpoint thread behind
        except Exception:
            pass
        self._unlock()

    def _unlock(self) -> None:
        if getattr(self, "wlock", None) is not None:
            self.wlock.release()


def run_job(model_dir: str, config: Dict[str, Any], datatype: str = "file",
            device: Optional[str] = None, ctx: Optional[DistContext] = None,
            backend: str = "auto", data: Optional[tuple] = None) -> Dict[str, Any]:
    """Train to ``config['iter']`` steps (resuming if a checkpoint exists).  Returns a
    summary dict.  Only rank 0 writes result/metrics/checkpoints."""
    job = JobRun(model_dir, config, datatype, device=device, ctx=ctx, backend=backend, data=data)
    try:
        while job.pending():
            job.before_step()
            job.step()
            if job.after_step():
                break
        return job.finish()
    except Exception as exc:
        job.fail(exc)
        raise


def _checkpoint(model_dir: str, eng: TrainEngine, chief: bool) -> None:
    state = ckpt.engine_state(eng)          # collective under the sharded "ps" strategy
    if chief:
        ckpt.save(model_dir, eng.host_step, state)


def _agree(ctx: DistContext, action: str) -> str:
    """Rank 0's control decision broadcast to all ranks (so every rank stops together)."""
    if not ctx.enabled:
        return action
    import torch.distributed as dist
    codes = {"": 0, "stop": 1, "pause": 2, "ckpt": 3}
    t = torch.tensor([codes.get(action, 0)], device=ctx.device)
    dist.broadcast(t, src=0)
    return {v: k for k, v in codes.items()}[int(t.item())]


def read_train_results(path: str, iters: int) -> Dict[str, Any]:
    """Reference monitor parse (apps/runtime/views.py:44-72).

    * ``every_result``: the leading run of ``step...`` lines, string values; the parse stops
      at the first line that is not a step line, as the reference's ``while`` does (:55);
    * ``final_accuracy`` is attached only when more than ``iter/100`` step rows exist (:66),
      and then it is the STRING after ``:`` on the line that ended the run (:70), or — if
      the file ended there — the float mean of the logged batch accuracies (:67-68).
    A stopper line without ``:`` (which would raise in the reference) falls back to the
    mean."""
    out: Dict[str, Any] = {"every_result": []}
    if not os.path.exists(path):
        return out
    accs = []
    stopper = ""
    with open(path) as f:
        for line in f:
            if not line.startswith("step"):
                stopper = line
                break
            parts = dict(p.split(":", 1) for p in line.split(",") if ":" in p)
            row = {"step": parts.get("step", ""), "accuracy": parts.get("accuracy", "").strip(),
                   "duration": parts.get("duration", "").strip()}
            out["every_result"].append(row)
            accs.append(float(row["accuracy"]))
    if len(accs) > int(iters) / 100:
        if len(stopper) < 1 or ":" not in stopper:
            out["final_accuracy"] = float(sum(accs)) / len(accs)
        else:
            out["final_accuracy"] = stopper.split(":")[1].strip()
    return out

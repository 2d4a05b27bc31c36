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


def run_job(model_dir: str, config: Dict[str, Any], datatype: str = "file",
            device: Optional[str] = None, ctx: Optional[DistContext] = None,
            backend: str = "auto", data: Optional[tuple] = None) -> Dict[str, Any]:
    """Train to ``config['iter']`` steps (resuming if a checkpoint exists).  Returns a
    summary dict.  Only rank 0 writes result/metrics/checkpoints."""
    ctx = ctx or DistContext()
    chief = ctx.is_chief
    cfg = parse_train_config(config)
    if device is None:
        device = str(ctx.device) if ctx.enabled else ("cuda" if torch.cuda.is_available() else "cpu")
    if chief:
        write_status(model_dir, state="running", pid=os.getpid(), device=device, world=ctx.world)
    train, test = data if data is not None else load_job_data(model_dir, datatype, cfg.ratio)
    eng = TrainEngine(cfg, train, device=device, ctx=ctx, backend=backend,
                      strategy=config.get("options", {}).get("strategy", "allreduce")
                      if isinstance(config.get("options"), dict) else "allreduce")
    last = ckpt.latest(model_dir)
    if last is not None:
        ckpt.restore_engine(eng, ckpt.load(last[1]))
    fault_at = int(os.environ.get("CSA_FAULT_AT_STEP", "-1"))     # raise (crash) at this step
    hang_at = int(os.environ.get("CSA_HANG_AT_STEP", "-1"))       # stop making progress (watchdog tests)
    result_path = os.path.join(model_dir, RESULT)
    metrics_path = os.path.join(model_dir, METRICS)
    log_every = max(1, cfg.log_every)
    t_int = time.perf_counter()
    int_start = eng.host_step
    state = "done"
    try:
        while eng.host_step < cfg.iter:
            step = eng.host_step
            if step == fault_at:
                raise RuntimeError(f"injected fault at step {step}")
            if step == hang_at:
                while True:
                    time.sleep(1.0)
            eng.step()
            if step % log_every != 0:
                continue
            # reference: the accuracy logged for step s is the batch of step s evaluated
            # with the pre-update weights — exactly this step's forward pass
            eng.sync_device()
            eng.sync.check()   # a timed-out peer-buffer collective fails the job
            now = time.perf_counter()
            n = eng.host_step - int_start
            step_time = (now - t_int) / max(n, 1)
            if chief:
                acc = eng.last_batch_accuracy()
                with open(result_path, "a") as f:
                    f.write("step:%d,accuracy:%f,duration:%f\n" % (step, acc, step_time))
                mm = eng.metrics_since(int_start)
                with open(metrics_path, "a") as f:
                    f.write(json.dumps({"step": step, "loss": mm["loss"], "accuracy": mm["accuracy"],
                                        "batch_accuracy": acc, "step_ms": step_time * 1e3,
                                        "samples_per_s": cfg.batch_size * ctx.world / max(step_time, 1e-9),
                                        "time": time.time()}) + "\n")
                write_status(model_dir, step=eng.host_step, heartbeat=time.time())   # watchdog liveness
            if cfg.ckpt_every > 0 and step > 0 and step % cfg.ckpt_every == 0:
                _checkpoint(model_dir, eng, chief)
            t_int, int_start = time.perf_counter(), eng.host_step
            action = _agree(ctx, read_control(model_dir) if chief else "")
            if action == "stop":
                state = "stopped"
                break
            if action == "pause":
                _checkpoint(model_dir, eng, chief)
                if chief:
                    write_status(model_dir, state="paused", step=eng.host_step)
                state = "paused"
                break
        eng.sync_device()
        final_acc = None
        if state == "done":
            final_acc = eng.evaluate(test) if len(test) else eng.last_batch_accuracy()
            if chief:
                with open(result_path, "a") as f:
                    f.write("final_accuracy:%f\n\n" % final_acc)
        if state != "paused":
            _checkpoint(model_dir, eng, chief)
        if chief:
            write_status(model_dir, state=state, step=eng.host_step, final_accuracy=final_acc,
                         backend=eng.backend, fallback=eng.fallback_reason)
        return {"state": state, "step": eng.host_step, "final_accuracy": final_acc, "backend": eng.backend}
    except Exception as exc:
        if chief:
            write_status(model_dir, state="failed", step=eng.host_step, error=repr(exc),
                         trace=traceback.format_exc()[-4000:])
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
    codes = {"": 0, "stop": 1, "pause": 2}
    t = torch.tensor([codes.get(action, 0)], device=ctx.device)
    dist.broadcast(t, src=0)
    return {v: k for k, v in codes.items()}[int(t.item())]


def read_train_results(path: str, iters: int) -> Dict[str, Any]:
    """Reference monitor parse (apps/runtime/views.py:44-72): ``every_result`` rows with
    string values; ``final_accuracy`` from the final line, or — once more than iter/100
    rows exist without one — the mean of the logged accuracies."""
    out: Dict[str, Any] = {"every_result": []}
    if not os.path.exists(path):
        return out
    final = None
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith("final_accuracy:"):
                final = float(line.split(":", 1)[1])
                continue
            parts = dict(p.split(":", 1) for p in line.split(",") if ":" in p)
            if {"step", "accuracy", "duration"} <= parts.keys():
                out["every_result"].append({"step": parts["step"], "accuracy": parts["accuracy"],
                                            "duration": parts["duration"]})
    rows = out["every_result"]
    if final is not None:
        out["final_accuracy"] = final
    elif rows and len(rows) > max(int(iters), 0) // 100:
        out["final_accuracy"] = float(np.mean([float(r["accuracy"]) for r in rows]))
    return out

"""Packed GPU host: one process per GPU that trains several single-GPU jobs at once.

``bench.py --jobs K`` measured (profiles/r2_multitenant.md) that K jobs as K separate
processes on one MI355X deliver LESS aggregate throughput than one job alone (the
contexts time-share the card), while K jobs replayed as K branches of ONE HIP graph in
one process deliver ~1.9x at K=4.  So the job manager (``runtime.jobs``, executor
``process`` with packing on) sends every single-GPU job placed on a GPU to that GPU's
host process instead of starting a worker per job:

    python -m cloud_server_amd.runtime.gpu_host --spool DIR --device cuda:0 [--backend B]

Protocol (files, so the manager never touches HIP and a host crash loses nothing but
its in-flight steps):
* ``DIR/inbox/<jid>.json``  — {"jid", "model_dir", "datatype"} posted by the manager;
* ``DIR/done/<jid>.json``   — {"jid", "rc"} written by the host when the job ends
  (rc 0: done / stopped / paused, status.json has the state; rc 1: failed);
* per-job control (stop / pause), heartbeats, metrics, checkpoints: exactly the files a
  single-job worker uses (``runtime.trainer.JobRun``).

Between packed steps the host admits new jobs and retires finished ones; the set of jobs
changing re-captures the packed graph (every engine keeps its state).  A new job is BUILT
on a builder thread (data decode, HBM upload, HIP program planning, its 2 warm-up steps,
on a stream of its own) while the hosted jobs keep stepping; only the re-capture stops
them (~10 ms, profiles/r3_multitenant.md).  Captures and builds never overlap.  A job whose step
raises fails alone; a fault that kills the process fails every job it hosted (the
manager's auto-restart policy then resumes them from their checkpoints).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import threading
import time
import traceback
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict, List

POLL_S = 0.05


def _post_done(spool: str, jid: int, rc: int) -> None:
    d = os.path.join(spool, "done")
    os.makedirs(d, exist_ok=True)
    tmp = os.path.join(d, f".{jid}.tmp")
    with open(tmp, "w") as f:
        json.dump({"jid": jid, "rc": rc, "time": time.time()}, f)
    os.replace(tmp, os.path.join(d, f"{jid}.json"))


def _take_inbox(spool: str) -> List[dict]:
    inbox = os.path.join(spool, "inbox")
    out = []
    try:
        names = sorted(os.listdir(inbox))
    except OSError:
        return out
    for n in names:
        if not n.endswith(".json"):
            continue
        p = os.path.join(inbox, n)
        try:
            with open(p) as f:
                req = json.load(f)
            os.remove(p)
        except (OSError, json.JSONDecodeError):
            continue                      # half-written: the manager renames atomically
        out.append(req)
    return out


def _build_job(req: dict, device: str, backend: str, lock: threading.Lock):
    """Construct (and warm up) one job off the stepping thread, on its own stream."""
    import torch
    from .trainer import JobRun
    with open(os.path.join(req["model_dir"], "model.json"), encoding="utf-8") as f:
        config = json.load(f)
    cuda = device.startswith("cuda") and torch.cuda.is_available()
    with lock:                                   # never while the stepping thread captures
        s = torch.cuda.Stream(torch.device(device)) if cuda else None
        with (torch.cuda.stream(s) if s is not None else contextlib.nullcontext()):
            job = JobRun(req["model_dir"], config, req.get("datatype", "file"), device=device, backend=backend,
                         packed=True)
            if s is not None and job.eng.use_graph and job.pending():
                job.eng._warm_up(device_sync=False)   # the pack captures it without re-warming
            if s is not None:
                s.synchronize()
    return job


def _drain(device: str) -> None:
    """Wait until the device is idle.  Called before the host drops its last reference to a
    job's engine (retire / fail) or to the packed graph: the engine's blocks were allocated
    on its builder stream, and the caching allocator hands a freed block to the next user
    of that (pooled) stream without ordering it after the packed replay still reading it
    on the branch streams."""
    import torch
    if device.startswith("cuda") and torch.cuda.is_available():
        torch.cuda.synchronize(torch.device(device))


def serve(spool: str, device: str, backend: str = "auto", idle_exit_s: float = 0.0,
          parent_pid: int = 0) -> int:
    from .multijob import PackedJobs
    from .trainer import JobRun

    jobs: Dict[int, JobRun] = {}
    building: Dict[int, Future] = {}
    builder = ThreadPoolExecutor(max_workers=1, thread_name_prefix="csa-job-build")
    gpu_lock = threading.Lock()             # builds vs captures of the packed graph
    pack = None
    idle_since = time.time()
    parent = parent_pid or os.getppid()     # the manager's launcher; if it dies we are orphaned

    def retire(jid: int, rc: int) -> None:
        _drain(device)                      # nothing in flight still uses its memory
        jobs.pop(jid, None)
        _post_done(spool, jid, rc)

    while True:
        changed = False
        for req in _take_inbox(spool):
            jid = int(req["jid"])
            building[jid] = builder.submit(_build_job, req, device, backend, gpu_lock)
        for jid, fut in list(building.items()):
            if not fut.done():
                continue
            del building[jid]
            try:
                jobs[jid] = fut.result()
                changed = True
            except Exception:
                traceback.print_exc()
                _post_done(spool, jid, 1)
        # jobs with nothing left to run (resumed at their last step) end before stepping
        for jid, job in list(jobs.items()):
            if not job.pending():
                rc = _finish(job)
                retire(jid, rc)
                changed = True
        if os.getppid() != parent:
            # the manager is gone (killed without a clean shutdown): checkpoint and stop
            # every hosted job rather than keep a GPU context nobody can control
            for jid, fut in list(building.items()):
                try:
                    jobs[jid] = fut.result()
                except Exception:
                    _post_done(spool, jid, 1)
            for jid, job in list(jobs.items()):
                job.state = "stopped"
                retire(jid, _finish(job))
            builder.shutdown(wait=True)
            return 0
        if not jobs:
            pack = None
            if idle_exit_s and not building and time.time() - idle_since > idle_exit_s:
                builder.shutdown(wait=True)
                return 0
            time.sleep(POLL_S)
            continue
        idle_since = time.time()
        if changed or pack is None:
            pack = PackedJobs([j.eng for j in jobs.values()])
        failed = []
        for jid, job in jobs.items():
            try:
                job.before_step()
            except Exception as exc:
                job.fail(exc)
                failed.append(jid)
        for jid in failed:
            retire(jid, 1)
        if failed:
            continue                      # re-pack without them before stepping
        # 8 steps of every job in one multi-step graph launch when no job has a hook inside
        # them (PackedJobs.run_steps; 2.4x a lone job's throughput at 4 jobs)
        k = int(os.environ.get("CSA_GRAPH_STEPS", "32"))
        group = pack.graph is not None and k > 1 and all(j.groupable(k) for j in jobs.values())
        # a launch that may capture (new pack, first multi-step launch) waits for a build
        # in flight; plain replays run alongside it
        may_capture = pack.graph is None or (group and pack.graph_k is None)
        with (gpu_lock if may_capture else contextlib.nullcontext()):
            if group:
                pack.run_steps(k)
            else:
                pack.step()
        for jid, job in list(jobs.items()):
            try:
                end = job.after_step()
            except Exception as exc:
                job.fail(exc)
                retire(jid, 1)
                pack = None
                continue
            if end or not job.pending():
                retire(jid, _finish(job))
                pack = None


def _finish(job) -> int:
    try:
        job.finish()
        return 0
    except Exception as exc:
        job.fail(exc)
        return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cloud_server_amd.runtime.gpu_host")
    ap.add_argument("--spool", required=True)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--idle-exit", type=float, default=0.0,
                    help="exit after this many seconds without jobs (0: never)")
    ap.add_argument("--parent-pid", type=int, default=0,
                    help="the launcher's pid: the host stops its jobs and exits when it is gone")
    a = ap.parse_args(argv)
    os.makedirs(os.path.join(a.spool, "inbox"), exist_ok=True)
    os.makedirs(os.path.join(a.spool, "done"), exist_ok=True)
    return serve(a.spool, a.device, a.backend, a.idle_exit, a.parent_pid)


if __name__ == "__main__":
    sys.exit(main())

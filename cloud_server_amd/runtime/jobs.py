"""Job manager: queue, GPU-slot placement, launch, control and bookkeeping of training jobs.

Replaces the reference control plane — paramiko SSH into the cluster host, ``docker cp``
into fixed PS/worker containers, ``pkill -9 python``, ``nohup python ...`` (C15, C21,
C29; apps/construction/views.py:97-146) — with a local manager:

* a job = one ``model.json`` in ``NJUCloud/<uid>/model/<m>/`` plus a DB row whose state
  follows ``queued -> running -> (paused | stopped | failed | done)``;
* placement by the native GPU-slot scheduler (``runtime.scheduler``), several small jobs
  per GPU, data-parallel jobs over several GPUs;
* packing (``settings.pack_jobs``): the single-GPU jobs placed on one GPU all run in that
  GPU's host process (``runtime.gpu_host``) as branches of one HIP graph — measured
  ~1.9x aggregate at 4 jobs, where 4 separate processes lose throughput
  (profiles/r2_multitenant.md);
* executors: ``process`` (default; one worker process per rank, started by a launcher
  process that is spawned before this process touches the GPU, so no process that
  initialised HIP ever forks/execs), ``thread`` and ``inline`` (tests, CPU);
* control: stop / pause write ``control.json`` (the trainer checks it every log
  interval and checkpoints on pause); resume re-queues the job and the trainer restores
  the newest checkpoint; a worker that dies is marked failed (its slots are released)
  and can be resumed the same way;
* recovery policy: a worker that fails AFTER making progress (a newer checkpoint than
  the one it started from) is re-queued automatically, up to ``max_restarts`` times
  (``CSA_MAX_RESTARTS``, default 2), and resumes from that checkpoint; a failure without
  progress (bad data, a deterministic crash) ends the job as ``failed`` at once.
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import queue
import signal
import socket
import subprocess
import sys
import threading
import time
import traceback
from typing import Any, Dict, List, Optional

from ..store.db import Database
from ..utils.locks import SUBMIT_LOCK, locked
from . import checkpoint as ckpt
from .scheduler import make_scheduler
from .trainer import CONTROL, STATUS, run_job, write_status

TERMINAL = ("done", "stopped", "failed", "paused", "resumed")
ACTIVE = ("queued", "running")


class JobConflict(ValueError):
    """A job for this (user, model) is already queued or running (HTTP 409)."""


def _launcher_main(req: "mp.Queue", resp: "mp.Queue") -> None:   # pragma: no cover - subprocess
    """Runs in a spawned helper that never initialises HIP: owns every worker Popen."""
    procs: Dict[int, subprocess.Popen] = {}
    kill_at: Dict[int, float] = {}          # SIGTERM sent; SIGKILL the group after a grace period
    while True:
        try:
            msg = req.get(timeout=0.2)
        except queue.Empty:
            msg = None
        if msg is not None:
            kind = msg[0]
            if kind == "launch":
                _, jid, argv, env, cwd, log = msg
                with open(log, "ab") as lf:
                    procs[jid] = subprocess.Popen(argv, env=env, cwd=cwd, stdout=lf, stderr=subprocess.STDOUT,
                                                  start_new_session=True)
            elif kind == "kill":
                p = procs.get(msg[1])
                if p is not None and p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)     # the worker's own session/group
                    except OSError:
                        p.terminate()
                    kill_at[msg[1]] = time.time() + 15.0
            elif kind == "exit":
                for p in procs.values():
                    if p.poll() is None:
                        p.terminate()
                return
        for jid, t in list(kill_at.items()):
            p = procs.get(jid)
            if p is None or p.poll() is not None:
                kill_at.pop(jid, None)
            elif time.time() > t:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    p.kill()
                kill_at.pop(jid, None)
        for jid, p in list(procs.items()):
            rc = p.poll()
            if rc is not None:
                resp.put(("exited", jid, rc))
                del procs[jid]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class JobManager:
    def __init__(self, settings, db: Database, executor: Optional[str] = None,
                 ngpu: Optional[int] = None, slots_per_gpu: Optional[int] = None):
        self.settings = settings
        self.db = db
        self.executor = executor or settings.executor
        if ngpu is None:
            ngpu = self._count_gpus()
        self.ngpu = ngpu
        self.use_cpu = ngpu == 0
        if slots_per_gpu is None:
            slots_per_gpu = int(getattr(settings, "slots_per_gpu", 0) or 1)
        self.pack = bool(getattr(settings, "pack_jobs", False)) and self.executor == "process"
        self.slots_per_gpu = slots_per_gpu
        self.sched = make_scheduler(max(ngpu, 1), slots_per_gpu if ngpu else 2)
        self.hosts: Dict[int, Dict[str, Any]] = {}     # packed host per GPU: spool, alive, jobs
        self.max_restarts = int(os.environ.get("CSA_MAX_RESTARTS", "2"))
        self.running: Dict[int, Dict[str, Any]] = {}
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._launcher = None
        if self.executor == "process":
            ctx = mp.get_context("spawn")
            self._req, self._resp = ctx.Queue(), ctx.Queue()
            self._launcher = ctx.Process(target=_launcher_main, args=(self._req, self._resp), daemon=True)
            self._launcher.start()
        self._thread = threading.Thread(target=self._loop, name="csa-jobs", daemon=True)
        self._thread.start()
        self._recover()

    @staticmethod
    def _count_gpus() -> int:
        vis = os.environ.get("CSA_GPUS")
        if vis:
            return len([x for x in vis.split(",") if x.strip()])
        try:
            import torch
            return torch.cuda.device_count()   # does not initialise HIP on this image
        except Exception:
            return 0

    SERVE_JOB = -1000          # scheduler owner id of the API process's serving slots

    def reserve_serving(self, gpu: int) -> int:
        """Take ``settings.serve_slots`` slots of GPU ``gpu`` for the API process (its
        resident inference graphs and GPU preprocessing share that GPU with training), so
        least-loaded placement steers jobs elsewhere.  Never takes a GPU's last slot, counting
        the jobs already placed there: a reservation that would fill the GPU is undone.  Each
        slot has its own owner id (``SERVE_JOB - i``), so ``release_serving`` frees them all.
        Returns the number of slots reserved."""
        n = int(getattr(self.settings, "serve_slots", 1) or 0)
        if self.use_cpu or not 0 <= gpu < self.ngpu:
            return 0
        got = []
        with self._lock:
            for i in range(n):
                owner = self.SERVE_JOB - len(getattr(self, "serve_owners", [])) - i
                if not self.sched.reserve(owner, gpu):
                    break
                if self.sched.load(gpu) >= self.slots_per_gpu:     # that was the last slot
                    self.sched.release(owner)
                    break
                got.append(owner)
            self.serve_owners = getattr(self, "serve_owners", []) + got
        self.serve_reserved = (gpu, len(got))
        return len(got)

    def release_serving(self) -> int:
        """Free every serving slot this manager reserved."""
        with self._lock:
            owners, self.serve_owners = getattr(self, "serve_owners", []), []
        return sum(self.sched.release(o) for o in owners)

    # ------------------------------------------------------------------ public API
    def submit(self, owner: int, model: str, datatype: str, config: Dict[str, Any],
               ngpus: int = 1, resume_of: Optional[int] = None) -> int:
        """Queue a job for (owner, model).  One job per model dir at a time: a queued or
        running job makes this raise ``JobConflict`` (the reference instead ``pkill``ed
        whatever ran, apps/construction/views.py:128-129); a paused one is superseded
        (marked ``stopped``) unless this call resumes it (``resume_of``: then it is marked
        ``resumed``).  The check and the insert run under the model dir's submit lock, so
        concurrent API workers cannot both admit a job."""
        mdir = self.settings.model_dir(owner, model)
        os.makedirs(mdir, exist_ok=True)
        with locked(os.path.join(mdir, SUBMIT_LOCK)):
            prior = [j for j in self.db.jobs_for(owner, model) if j["state"] in ACTIVE + ("paused",)]
            busy = [j["id"] for j in prior if j["state"] in ACTIVE]
            if busy:
                raise JobConflict(f"model {model!r} already has job {busy[-1]} "
                                  f"({self.db.get_job(busy[-1])['state']}): stop it first")
            with open(os.path.join(mdir, "model.json"), "w", encoding="utf-8") as f:
                json.dump(config, f, ensure_ascii=False)
            try:
                os.remove(os.path.join(mdir, CONTROL))
            except OSError:
                pass
            jid = self.db.add_job(owner, model, datatype, config)
            for j in prior:                              # paused jobs of this model
                if j["id"] == resume_of:
                    self.db.update_job(j["id"], state="resumed", error=f"resumed as job {jid}")
                else:
                    self.db.update_job(j["id"], state="stopped", error=f"superseded by job {jid}")
            write_status(mdir, state="queued", job=jid)
        ngpus = max(1, min(int(ngpus), max(self.ngpu, 1)))
        if not self.sched.submit(jid, 1 if self.use_cpu else ngpus):
            self.db.update_job(jid, state="failed", error="cannot place job")
            raise ValueError("job needs more GPUs than the node has")
        with self._lock:
            self.running[jid] = {"owner": owner, "model": model, "mdir": mdir, "ngpus": ngpus,
                                 "datatype": datatype, "state": "queued"}
        if self.executor == "inline":
            self._admit()
        return jid

    def control(self, jid: int, action: str) -> Dict[str, Any]:
        job = self.db.get_job(jid)
        if job is None:
            raise KeyError(jid)
        mdir = self.settings.model_dir(job["owner_id"], job["model"])
        if action in ("stop", "pause"):
            if job["state"] == "queued":
                self.sched.cancel(jid)
                self._finish(jid, "stopped" if action == "stop" else "paused")
            else:
                with self._lock:
                    if jid in self.running:
                        self.running[jid]["user_stop"] = True
                with open(os.path.join(mdir, CONTROL), "w") as f:
                    json.dump({"action": action, "time": time.time()}, f)
            return {"job": jid, "action": action}
        if action == "resume":
            if job["state"] not in ("paused", "stopped", "failed"):
                raise ValueError(f"job {jid} is {job['state']}")
            cfg = json.loads(job["config"])
            return {"job": self.submit(job["owner_id"], job["model"], job["datatype"], cfg, resume_of=jid),
                    "action": "resume"}
        raise ValueError(f"unknown action {action!r}")

    def status(self, jid: int) -> Dict[str, Any]:
        job = self.db.get_job(jid)
        if job is None:
            raise KeyError(jid)
        mdir = self.settings.model_dir(job["owner_id"], job["model"])
        st = {}
        try:
            with open(os.path.join(mdir, STATUS)) as f:
                st = json.load(f)
        except (OSError, json.JSONDecodeError):
            pass
        out = {k: job[k] for k in ("id", "model", "datatype", "state", "created", "started", "finished", "gpu", "error")}
        out["progress"] = st
        return out

    def wait(self, jid: int, timeout: float = 300.0) -> str:
        t0 = time.time()
        while time.time() - t0 < timeout:
            j = self.db.get_job(jid)
            if j and j["state"] in TERMINAL:
                return j["state"]
            time.sleep(0.05)
        raise TimeoutError(f"job {jid} still {self.db.get_job(jid)['state']}")

    def shutdown(self) -> None:
        self._stop.set()
        if self._launcher is not None:
            try:
                self._req.put(("exit",))
                self._launcher.join(timeout=5)
            except Exception:
                pass

    # ------------------------------------------------------------------ internals
    def _recover(self) -> None:
        """Jobs left running by a previous server instance are marked failed (resumable)."""
        for j in self.db.active_jobs():
            if j["id"] not in self.running and j["state"] in ("queued", "running"):
                self.db.update_job(j["id"], state="failed", error="server restarted", finished=time.time())

    def _loop(self) -> None:
        last_watch = 0.0
        while not self._stop.is_set():
            try:
                self._admit()
                self._reap()
                if time.time() - last_watch > 2.0:
                    last_watch = time.time()
                    self._watchdog()
            except Exception:   # pragma: no cover - keep the dispatcher alive
                traceback.print_exc()
            time.sleep(0.05)

    def _watchdog(self) -> None:
        """Kill + fail a worker whose heartbeat (status.json, written at every log point)
        is older than ``settings.heartbeat_s`` — a hung collective or kernel, or a dead
        rank that left its peers blocked."""
        if self._launcher is None:
            return
        limit = float(getattr(self.settings, "heartbeat_s", 0) or 0)
        if limit <= 0:
            return
        now = time.time()
        with self._lock:
            items = [(jid, info) for jid, info in self.running.items() if info.get("state") == "running"]
        for jid, info in items:
            last = info.get("launched", now)
            try:
                with open(os.path.join(info["mdir"], STATUS)) as f:
                    st = json.load(f)
                last = max(last, float(st.get("heartbeat", 0)), float(st.get("updated", 0)))
            except (OSError, ValueError, json.JSONDecodeError):
                pass
            if now - last > limit and not info.get("killed"):
                info["killed"] = True
                info["kill_reason"] = f"no heartbeat for {now - last:.0f}s"
                # a packed job shares its host process: a hung host takes its jobs along
                self._req.put(("kill", self._host_id(info["host"]) if "host" in info else jid))

    def _admit(self) -> None:
        while True:
            nxt = self.sched.next()
            if nxt is None:
                return
            jid, gpus = nxt
            with self._lock:
                info = self.running.get(jid)
            if info is None:
                self.sched.release(jid)
                continue
            info["gpus"] = gpus
            info["state"] = "running"
            last = ckpt.latest(info["mdir"])
            info["ckpt_at_launch"] = last[0] if last else -1
            self.db.update_job(jid, state="running", started=time.time(),
                               gpu=",".join(map(str, gpus)) if not self.use_cpu else "cpu")
            self._launch(jid, info)

    def _launch(self, jid: int, info: Dict[str, Any]) -> None:
        mdir, datatype = info["mdir"], info["datatype"]
        with open(os.path.join(mdir, "model.json"), encoding="utf-8") as f:
            config = json.load(f)
        if self.executor in ("inline", "thread"):
            def body():
                rc = 0
                try:
                    dev = "cpu" if self.use_cpu else f"cuda:{info['gpus'][0]}"
                    run_job(mdir, config, datatype, device=dev, backend=self.settings.train_backend)
                except Exception:
                    rc = 1
                self._exited(jid, rc)
            if self.executor == "inline":
                body()
            else:
                threading.Thread(target=body, name=f"job-{jid}", daemon=True).start()
            return
        env = self._worker_env()
        n = len(info["gpus"])
        if self.pack and n == 1:
            self._launch_packed(jid, info, env)
            return
        if not self.use_cpu:
            env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, info["gpus"]))
        mod = ["-m", "cloud_server_amd.runtime.worker", "--model-dir", mdir, "--datatype", datatype,
               "--backend", self.settings.train_backend]
        if n > 1:
            port = _free_port()             # a fixed 29500 + jid formula collided
            argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                    "--master-addr", "127.0.0.1", "--master-port", str(port)] + mod   # -m: run as a module
        else:
            argv = [sys.executable] + mod + ["--device", "cpu" if self.use_cpu else "cuda:0"]
        env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")   # RCCL errors/timeouts abort the rank
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        info["launched"] = time.time()
        self._req.put(("launch", jid, argv, env, mdir, os.path.join(mdir, "worker.log")))

    def _worker_env(self) -> Dict[str, str]:
        env = dict(os.environ)
        env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__))))] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
        return env

    # ---- packed hosts: one process per GPU hosting its single-GPU jobs ----
    @staticmethod
    def _host_id(gpu: int) -> int:
        return -(gpu + 1)             # launcher process key (job ids are positive)

    def _launch_packed(self, jid: int, info: Dict[str, Any], env: Dict[str, str]) -> None:
        gpu = info["gpus"][0]
        with self._lock:
            h = self.hosts.get(gpu)
            if h is None or not h["alive"]:
                spool = os.path.join(self.settings.storage_root, "gpu_hosts", f"gpu{gpu}")
                os.makedirs(os.path.join(spool, "inbox"), exist_ok=True)
                os.makedirs(os.path.join(spool, "done"), exist_ok=True)
                # a previous host's unread inbox entries belong to jobs that were failed as
                # its orphans: never let the new host train them behind the manager's back
                inbox = os.path.join(spool, "inbox")
                for n in os.listdir(inbox):
                    try:
                        os.remove(os.path.join(inbox, n))
                    except OSError:
                        pass
                h = {"spool": spool, "alive": True, "jobs": set()}
                self.hosts[gpu] = h
                if not self.use_cpu:
                    env["HIP_VISIBLE_DEVICES"] = str(gpu)
                env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
                argv = [sys.executable, "-m", "cloud_server_amd.runtime.gpu_host", "--spool", spool,
                        "--device", "cpu" if self.use_cpu else "cuda:0",
                        "--backend", self.settings.train_backend, "--parent-pid", str(self._launcher.pid)]
                self._req.put(("launch", self._host_id(gpu), argv, env, spool, os.path.join(spool, "host.log")))
            h["jobs"].add(jid)
            info["host"] = gpu
            info["launched"] = time.time()
            inbox = os.path.join(h["spool"], "inbox")
            tmp = os.path.join(inbox, f".{jid}.tmp")
            with open(tmp, "w") as f:
                json.dump({"jid": jid, "model_dir": info["mdir"], "datatype": info["datatype"]}, f)
            os.replace(tmp, os.path.join(inbox, f"{jid}.json"))

    def _poll_hosts(self) -> None:
        with self._lock:
            hosts = list(self.hosts.items())
        for gpu, h in hosts:
            d = os.path.join(h["spool"], "done")
            try:
                names = [n for n in os.listdir(d) if n.endswith(".json")]
            except OSError:
                continue
            for n in names:
                p = os.path.join(d, n)
                try:
                    with open(p) as f:
                        rec = json.load(f)
                    os.remove(p)
                except (OSError, json.JSONDecodeError):
                    continue
                jid = int(rec["jid"])
                with self._lock:
                    h["jobs"].discard(jid)
                self._exited(jid, int(rec.get("rc", 1)))

    def _host_exited(self, hid: int, rc: int) -> None:
        gpu = -hid - 1
        self._poll_hosts()                          # jobs that ended cleanly first
        with self._lock:
            h = self.hosts.get(gpu)
            if h is None:
                return
            h["alive"] = False
            orphans = list(h["jobs"])
            h["jobs"].clear()
            for jid in orphans:                     # posted but never admitted by the dead host
                try:
                    os.remove(os.path.join(h["spool"], "inbox", f"{jid}.json"))
                except OSError:
                    pass
        for jid in orphans:                         # the host died under them
            with self._lock:
                info = self.running.get(jid)
            if info is not None and not info.get("kill_reason"):
                info["kill_reason"] = f"gpu host exit code {rc}"
            self._exited(jid, rc or 1)

    def _reap(self) -> None:
        if self._launcher is None:
            return
        self._poll_hosts()
        while True:
            try:
                _, jid, rc = self._resp.get_nowait()
            except queue.Empty:
                return
            if jid < 0:
                self._host_exited(jid, rc)
            else:
                self._exited(jid, rc)

    def _exited(self, jid: int, rc: int) -> None:
        with self._lock:
            info = self.running.get(jid)
        mdir = info["mdir"] if info else None
        state = "failed"
        if mdir:
            try:
                with open(os.path.join(mdir, STATUS)) as f:
                    s = json.load(f).get("state")
                if rc == 0 and s in ("done", "stopped", "paused"):
                    state = s
            except (OSError, json.JSONDecodeError):
                pass
        err = None
        if state == "failed":
            err = (info or {}).get("kill_reason") or f"worker exit code {rc}"
            if info is not None and self._auto_restart(jid, info, err):
                return
        self._finish(jid, state, err)

    def _auto_restart(self, jid: int, info: Dict[str, Any], err: str) -> bool:
        """Re-queue a failed job that made progress since its launch (bounded)."""
        if info.get("user_stop") or info.get("restarts", 0) >= self.max_restarts:
            return False
        last = ckpt.latest(info["mdir"])
        if last is None or last[0] <= info.get("ckpt_at_launch", -1):
            return False
        self.sched.release(jid)
        info["restarts"] = info.get("restarts", 0) + 1
        info["state"] = "queued"
        info.pop("killed", None)
        info.pop("kill_reason", None)
        write_status(info["mdir"], state="queued", restarts=info["restarts"], last_error=err)
        self.db.update_job(jid, state="queued", error=f"restart {info['restarts']} after: {err}")
        if not self.sched.submit(jid, 1 if self.use_cpu else info["ngpus"]):
            return False
        if self.executor == "inline":
            self._admit()
        return True

    def _finish(self, jid: int, state: str, error: Optional[str] = None) -> None:
        self.sched.release(jid)
        with self._lock:
            info = self.running.pop(jid, None)
        if info and state in ("failed", "stopped", "paused"):
            write_status(info["mdir"], state=state)
        if info and info.get("restarts") and error is None:
            error = f"recovered after restart {info['restarts']}"
        self.db.update_job(jid, state=state, finished=time.time(), error=error)

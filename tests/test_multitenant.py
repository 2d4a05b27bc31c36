"""Multi-tenant packing (SURVEY §2.3 "multi-tenant job parallelism"; the reference ran one
job cluster-wide and killed the previous one, apps/construction/views.py:128-129):

* ``PackedJobs`` steps K independent engines as branches of one graph — every job's
  parameters after N packed steps equal those of the same job trained alone;
* ``runtime.gpu_host`` hosts several jobs in one process: concurrent jobs finish with the
  single-job result files, a failing job fails alone, an injected fault recovers through
  the manager's auto-restart, and the host retires jobs as they end;
* ``bench.py --jobs K`` prints one aggregate JSON line (GPU curve: scripts/gpu_pack.sh).
"""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

from cloud_server_amd.config import Settings
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine
from cloud_server_amd.runtime.jobs import JobManager
from cloud_server_amd.runtime.multijob import PackedJobs
from cloud_server_amd.runtime.trainer import RESULT, STATUS, read_train_results
from cloud_server_amd.store.db import Database

from test_runtime import SMALL, _prep_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(seed, opt="AdamOptimizer", device="cpu", backend="torch"):
    cfg = parse_train_config(dict(SMALL, optimizer_name=opt, options=dict(SMALL["options"], seed=seed)))
    return TrainEngine(cfg, synthetic_mnist(200, seed=seed), device=device, backend=backend)


def test_packed_jobs_match_solo_runs():
    solo = [_engine(s, o) for s, o in ((1, "AdamOptimizer"), (2, "AdagradOptimizer"))]
    for e in solo:
        for _ in range(6):
            e.step()
    packed = [_engine(s, o) for s, o in ((1, "AdamOptimizer"), (2, "AdagradOptimizer"))]
    pack = PackedJobs(packed)
    for _ in range(6):
        pack.step()
    assert pack.host_step == 6 and all(e.host_step == 6 for e in packed)
    assert pack.samples_per_step == 2 * 16
    for a, b in zip(solo, packed):
        torch.testing.assert_close(a.flat, b.flat, rtol=0, atol=0)
        torch.testing.assert_close(a.slots, b.slots, rtol=0, atol=0)


def test_packed_jobs_reject_mixed_devices_and_empty():
    with pytest.raises(ValueError):
        PackedJobs([])


def _settings(tmp_path):
    return Settings(storage_root=str(tmp_path / "s"), db_path=str(tmp_path / "db.sqlite3"),
                    executor="process", train_backend="torch", pack_jobs=True)


def test_gpu_host_runs_concurrent_jobs(tmp_path):
    s = _settings(tmp_path)
    assert s.slots_per_gpu == 4
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor="process", ngpu=0)
    try:
        assert jm.pack
        mdirs = [_prep_model(s, uid, f"m{i}", n=60) for i in range(2)]
        jids = [jm.submit(uid, f"m{i}", "file", dict(SMALL, iter=20 + 10 * i)) for i in range(2)]
        bad = jm.submit(uid, "empty", "file", dict(SMALL, iter=5))      # no data: fails alone
        assert jm.wait(bad, 300) == "failed"
        for i, (jid, mdir) in enumerate(zip(jids, mdirs)):
            log = os.path.join(s.storage_root, "gpu_hosts", "gpu0", "host.log")
            assert jm.wait(jid, 300) == "done", open(log).read() if os.path.exists(log) else jm.status(jid)
            st = json.load(open(os.path.join(mdir, STATUS)))
            assert st["state"] == "done" and st["step"] == 20 + 10 * i
            res = read_train_results(os.path.join(mdir, RESULT), 20 + 10 * i)
            assert len(res["every_result"]) == 3 + i and "final_accuracy" in res   # + the step == iter row
        # all of them were hosted by ONE process
        pids = {json.load(open(os.path.join(m, STATUS)))["pid"] for m in mdirs}
        assert len(pids) == 1
    finally:
        jm.shutdown()


def test_gpu_host_fault_recovers_via_auto_restart(tmp_path, monkeypatch):
    s = _settings(tmp_path)
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    monkeypatch.setenv("CSA_FAULT_AT_STEP", "25")
    monkeypatch.setenv("CSA_FAULT_ONCE", "1")
    jm = JobManager(s, db, executor="process", ngpu=0)
    try:
        mdir = _prep_model(s, uid, "m", n=60)
        jid = jm.submit(uid, "m", "file", dict(SMALL, iter=30))
        t0 = time.time()
        while time.time() - t0 < 240 and db.get_job(jid)["state"] not in ("done", "failed"):
            time.sleep(0.05)
        assert db.get_job(jid)["state"] == "done", db.get_job(jid)
        assert "restart 1" in (db.get_job(jid)["error"] or "")
        assert json.load(open(os.path.join(mdir, STATUS)))["step"] == 30
    finally:
        jm.shutdown()


def test_bench_jobs_flag_prints_aggregate_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--jobs", "2", "--steps", "2",
                          "--warmup", "1", "--batch", "8"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["metric"] == "train_samples_per_s" and d["config"]["jobs"] == 2
    assert d["config"]["global_batch"] == 16 and d["value"] > 0


def test_gpu_host_exits_when_orphaned(tmp_path):
    """A host whose parent (the manager's launcher) died stops its jobs and exits."""
    spool = tmp_path / "spool"
    code = ("import os, sys, subprocess, time\n"
            f"p = subprocess.Popen([sys.executable, '-m', 'cloud_server_amd.runtime.gpu_host', '--spool', r'{spool}',"
            " '--device', 'cpu', '--backend', 'torch', '--parent-pid', str(os.getpid())], cwd=r'" + ROOT + "',"
            " stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, stdin=subprocess.DEVNULL)\n"
            "print(p.pid, flush=True)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT)
    pid = int(out.stdout.strip().splitlines()[-1])
    t0 = time.time()
    def alive():
        try:
            with open(f"/proc/{pid}/stat") as f:
                return f.read().split(")")[-1].split()[0] != "Z"    # a zombie has exited
        except OSError:
            return False
    while time.time() - t0 < 60:
        if not alive():
            break
        time.sleep(0.2)
    else:
        os.kill(pid, 9)
        raise AssertionError("orphaned gpu_host kept running")


def test_gpu_host_drains_before_dropping_a_failed_job(tmp_path, monkeypatch):
    """a job failing in after_step is dropped only after the device is
    idle — its engine memory came from a pooled builder stream, so freeing it while the
    last packed replay still runs would let the next build reuse live memory."""
    import gc
    import weakref
    from cloud_server_amd.runtime import gpu_host
    from cloud_server_amd.runtime.trainer import JobRun
    s = _settings(tmp_path)
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    spool = tmp_path / "spool"
    (spool / "inbox").mkdir(parents=True)
    mdirs = [_prep_model(s, uid, f"m{i}", n=40) for i in range(2)]
    for i, m in enumerate(mdirs):
        with open(os.path.join(m, "model.json"), "w") as f:
            json.dump(dict(SMALL, iter=12), f)
        with open(spool / "inbox" / f"{i}.json", "w") as f:
            json.dump({"jid": i, "model_dir": m, "datatype": "file"}, f)
    engines = {}
    calls = {"n": 0}
    orig = JobRun.after_step

    def after_step(self):
        engines.setdefault(self.model_dir, weakref.ref(self.eng))
        if self.model_dir == mdirs[0] and self.eng.host_step >= 3:
            raise RuntimeError("injected after_step failure")
        return orig(self)

    drains = []

    def drain(device):
        gc.collect()
        ref = engines.get(mdirs[0])
        drains.append(ref is not None and ref() is not None)   # the failed engine still alive

    monkeypatch.setattr(JobRun, "after_step", after_step)
    monkeypatch.setattr(gpu_host, "_drain", drain)
    assert gpu_host.serve(str(spool), "cpu", "torch", idle_exit_s=0.3) == 0
    done = {int(n.split(".")[0]): json.load(open(spool / "done" / n))["rc"] for n in os.listdir(spool / "done")}
    assert done == {0: 1, 1: 0}
    assert drains and drains[0] is True          # drained while the failed job was still referenced

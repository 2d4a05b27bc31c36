"""Store, GPU-slot scheduler (native C++ vs Python policy), checkpoint/resume, trainer
(result.txt contract, control, fault injection), job manager executors and the warm
inference cache — all on CPU.

Reference behaviour pinned here: result.txt line format and the monitor's mean fallback
(construct_distribute.py:405-420, apps/runtime/views.py:44-72); Supervisor-style resume
from the newest checkpoint (:385-392); inference image prep (construct_inference.py:312-330)."""
import io
import json
import os
import random
import time

import numpy as np
import pytest
import torch
from PIL import Image

from cloud_server_amd.config import Settings
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.runtime import checkpoint as ckpt
from cloud_server_amd.runtime.jobs import JobManager
from cloud_server_amd.runtime.scheduler import NativeScheduler, PyScheduler
from cloud_server_amd.runtime.trainer import (CONTROL, RESULT, STATUS, read_train_results, run_job)
from cloud_server_amd.serve.inference import InferenceService, prepare_reference
from cloud_server_amd.store.db import Database, check_password, hash_password

SMALL = {"iter": 30, "learning_rate": 0.05, "ratio": 0.8, "loss_name": "entropy",
         "optimizer_name": "AdamOptimizer",
         "options": {"log_every": 10, "ckpt_every": 10, "batch_size": 16},
         "net_config": {"middle_layer": [{"layer": "conv", "filter": [3, 3, 4]},
                                         {"layer": "active", "active_func": "relu"},
                                         {"layer": "pool"},
                                         {"layer": "connect", "hidden": 16}]}}


def _data(n=400):
    ds = synthetic_mnist(n, seed=0)
    return ds.split(0.8)


# ---------------------------------------------------------------- store
def test_db_users_tokens_data_jobs(tmp_path):
    db = Database(str(tmp_path / "x.db"))
    uid = db.create_user("u1", "pw-12345678", "u1@x")
    assert check_password("pw-12345678", db.get_user(uid)["password"])
    assert not check_password("nope", db.get_user(uid)["password"])
    assert hash_password("a") != hash_password("a")          # salted
    k = db.token_for(uid)
    assert db.token_for(uid) == k and db.user_for_token(k)["id"] == uid
    db.delete_token(uid)
    assert db.user_for_token(k) is None
    pk = db.add_raw_data(uid, "NJUCloud/1/data/doc/a.csv", "doc")
    assert db.list_raw_data(uid)[0]["id"] == pk
    assert db.delete_raw_data(pk) and db.get_raw_data(pk) is None
    jid = db.add_job(uid, "m", "file", {"iter": 1})
    db.update_job(jid, state="running")
    assert [j["id"] for j in db.active_jobs()] == [jid]
    tok = db.new_reset_token(uid)
    assert db.use_reset_token(uid, tok) and not db.use_reset_token(uid, tok)
    with pytest.raises(Exception):
        db.create_user("u1", "x")


# ---------------------------------------------------------------- scheduler
def test_native_scheduler_matches_python_policy():
    rnd = random.Random(0)
    nat, py = NativeScheduler(4, 2, max_skip=3), PyScheduler(4, 2, max_skip=3)
    running = []
    jid = 0
    for _ in range(400):
        r = rnd.random()
        if r < 0.45:
            jid += 1
            n = rnd.choice([1, 1, 1, 2, 4])
            assert nat.submit(jid, n) == py.submit(jid, n)
        elif r < 0.75:
            a, b = nat.next(), py.next()
            assert (a is None and b is None) or (a[0] == b[0] and list(a[1]) == list(b[1])), (a, b)
            if a:
                running.append(a[0])
        elif r < 0.95 and running:
            j = running.pop(rnd.randrange(len(running)))
            assert nat.release(j) == py.release(j)
        else:
            j = rnd.randint(1, max(jid, 1))
            assert nat.cancel(j) == py.cancel(j)
        assert [nat.load(g) for g in range(4)] == [py.load(g) for g in range(4)]
        assert nat.queued() == py.queued()
    assert not nat.submit(999, 5)          # more GPUs than exist


def test_scheduler_packs_least_loaded_and_bounds_skips():
    s = NativeScheduler(2, 2, max_skip=1)
    for j in (1, 2, 3):
        s.submit(j, 1)
    assert s.next() == (1, [0]) and s.next() == (2, [1]) and s.next() == (3, [0])
    s.submit(4, 2)            # needs both GPUs; GPU 0 has 2 jobs, GPU 1 has 1
    s.submit(5, 1)
    assert s.next() == (5, [1])            # 5 may skip past 4 once
    s.release(1)
    s.submit(6, 1)
    assert s.next() is None                # 4 was skipped max_skip times: it now blocks 6
    s.release(2); s.release(3); s.release(5)
    assert s.next() == (4, [0, 1])


# ---------------------------------------------------------------- trainer / checkpoint
def test_run_job_result_contract_and_resume(tmp_path):
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    data = _data()
    out = run_job(mdir, SMALL, device="cpu", backend="torch", data=data)
    assert out["state"] == "done" and out["step"] == 30
    lines = open(os.path.join(mdir, RESULT)).read().splitlines()
    # rows 0, 10, 20 and the reference's row at step == iter (its loop logs it), then the
    # final line: iter/100 + 1 rows, as the monitor's gate expects (views.py:66)
    assert [l.split(",")[0] for l in lines[:4]] == ["step:0", "step:10", "step:20", "step:30"]
    assert lines[4].startswith("final_accuracy:") and lines[5] == ""
    res = read_train_results(os.path.join(mdir, RESULT), 30)
    assert len(res["every_result"]) == 4 and isinstance(res["final_accuracy"], str)   # views.py:70
    assert float(res["final_accuracy"]) == pytest.approx(out["final_accuracy"], abs=1e-6)
    last = ckpt.latest(mdir)
    assert last[0] == 30
    obj = torch.load(last[1], weights_only=True)                 # safe loader works
    assert obj["host_step"] == 30 and "layers.0.weight" in obj["model"]
    # extend the job: resumes at 30, runs to 50
    cfg2 = dict(SMALL, iter=50)
    out2 = run_job(mdir, cfg2, device="cpu", backend="torch", data=data)
    assert out2["step"] == 50
    steps = [r["step"] for r in read_train_results(os.path.join(mdir, RESULT), 50)["every_result"]]
    assert steps == ["0", "10", "20", "30", "40", "50"]     # resumed at 30: rows >= 30 re-logged once


def test_fault_injection_then_resume(tmp_path, monkeypatch):
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    data = _data()
    monkeypatch.setenv("CSA_FAULT_AT_STEP", "25")
    with pytest.raises(RuntimeError):
        run_job(mdir, SMALL, device="cpu", backend="torch", data=data)
    st = json.load(open(os.path.join(mdir, STATUS)))
    assert st["state"] == "failed" and "injected" in st["error"]
    assert ckpt.latest(mdir)[0] == 21            # checkpoint taken after step 20
    monkeypatch.delenv("CSA_FAULT_AT_STEP")
    out = run_job(mdir, SMALL, device="cpu", backend="torch", data=data)
    assert out["state"] == "done" and out["step"] == 30


def test_resume_is_exact(tmp_path):
    """Stopping at a checkpoint and resuming gives the same weights as an unbroken run
    (same optimizer slots and step count; the batch stream seeks to the same position)."""
    data = _data()
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a); os.makedirs(b)
    run_job(a, dict(SMALL, iter=33), device="cpu", backend="torch", data=data)
    o1 = ckpt.load(ckpt.latest(a)[1])
    run_job(b, dict(SMALL, iter=14), device="cpu", backend="torch", data=data)    # resumed part crosses an epoch
    run_job(b, dict(SMALL, iter=33), device="cpu", backend="torch", data=data)
    o2 = ckpt.load(ckpt.latest(b)[1])
    assert o1["host_step"] == o2["host_step"] == 33
    for k in o1["model"]:
        torch.testing.assert_close(o1["model"][k], o2["model"][k])     # deterministic on CPU
    torch.testing.assert_close(o1["slots"], o2["slots"])


def test_stop_and_pause_control(tmp_path):
    data = _data()
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    with open(os.path.join(mdir, CONTROL), "w") as f:
        json.dump({"action": "pause"}, f)
    out = run_job(mdir, dict(SMALL, iter=1000), device="cpu", backend="torch", data=data)
    assert out["state"] == "paused" and out["step"] == 1     # stops at the first log point
    assert ckpt.latest(mdir)[0] == 1
    os.remove(os.path.join(mdir, CONTROL))
    with open(os.path.join(mdir, CONTROL), "w") as f:
        json.dump({"action": "stop"}, f)
    out = run_job(mdir, dict(SMALL, iter=1000), device="cpu", backend="torch", data=data)
    assert out["state"] == "stopped" and out["step"] == 11


def test_monitor_mean_fallback(tmp_path):
    p = tmp_path / "result.txt"
    p.write_text("".join(f"step:{s},accuracy:{a},duration:0.1\n" for s, a in
                         [(0, 0.1), (100, 0.3), (200, 0.5)]))
    r = read_train_results(str(p), 100)          # > iter/100 rows, no final line -> mean
    assert r["final_accuracy"] == pytest.approx(0.3)
    r = read_train_results(str(p), 1000)
    assert "final_accuracy" not in r
    assert read_train_results(str(tmp_path / "none.txt"), 10) == {"every_result": []}


def test_monitor_final_line_gated_and_string(tmp_path):
    """views.py:55-70: the final line's value is returned as a string, and only when more
    than iter/100 rows were logged; the parse stops at the first non-step line."""
    p = tmp_path / "result.txt"
    body = "".join(f"step:{s},accuracy:{a},duration:0.1\n" for s, a in [(0, 0.1), (100, 0.3)])
    p.write_text(body + "final_accuracy:0.912000\n\n")
    r = read_train_results(str(p), 100)                    # 2 > 1: gated in
    assert r["final_accuracy"] == "0.912000"
    r = read_train_results(str(p), 200)                    # 2 > 2 is false: gated out
    assert "final_accuracy" not in r and len(r["every_result"]) == 2
    # a step line after a non-step line is not read (the reference's while loop stops)
    p.write_text(body + "final_accuracy:0.5\nstep:300,accuracy:0.9,duration:0.1\n")
    r = read_train_results(str(p), 0)
    assert [x["step"] for x in r["every_result"]] == ["0", "100"] and r["final_accuracy"] == "0.5"


# ---------------------------------------------------------------- job manager
def _settings(tmp_path, executor):
    return Settings(storage_root=str(tmp_path / "s"), db_path=str(tmp_path / "db.sqlite3"),
                    executor=executor, train_backend="torch")


def _prep_model(s, uid, name, n=120):
    mdir = s.model_dir(uid, name)
    os.makedirs(os.path.join(mdir, "data"), exist_ok=True)
    ds = synthetic_mnist(n, seed=4)
    tags = {}
    for i in range(n):
        fn = f"d{i}.png"
        Image.fromarray(ds.images[i].reshape(28, 28)).save(os.path.join(mdir, "data", fn))
        tags[fn] = str(int(ds.labels[i]))
    json.dump(tags, open(os.path.join(mdir, "tag.json"), "w"))
    return mdir


@pytest.mark.parametrize("executor", ["thread", "process"])
def test_job_manager_executors(tmp_path, executor):
    s = _settings(tmp_path, executor)
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor=executor, ngpu=0)
    try:
        mdir = _prep_model(s, uid, "m")
        jid = jm.submit(uid, "m", "file", dict(SMALL, iter=20))
        assert jm.wait(jid, 300) == "done", open(os.path.join(mdir, "worker.log")).read() \
            if os.path.exists(os.path.join(mdir, "worker.log")) else jm.status(jid)
        st = jm.status(jid)
        assert st["progress"]["state"] == "done" and st["progress"]["step"] == 20
        assert len(read_train_results(os.path.join(mdir, RESULT), 20)["every_result"]) == 3   # 0, 10, 20
        # a failing job is marked failed and can be resumed
        bad = jm.submit(uid, "empty", "file", dict(SMALL, iter=5))
        assert jm.wait(bad, 300) == "failed"
        with pytest.raises(ValueError):
            jm.control(jid, "resume")                        # done jobs cannot resume
    finally:
        jm.shutdown()


def test_job_pause_resume_thread(tmp_path):
    s = _settings(tmp_path, "thread")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor="thread", ngpu=0)
    try:
        mdir = _prep_model(s, uid, "m")
        cfg = dict(SMALL, iter=4000, options=dict(SMALL["options"], log_every=5))
        jid = jm.submit(uid, "m", "file", cfg)
        t0 = time.time()
        while not os.path.exists(os.path.join(mdir, RESULT)) and time.time() - t0 < 120:
            time.sleep(0.05)
        jm.control(jid, "pause")
        assert jm.wait(jid, 120) == "paused"
        step_at_pause = ckpt.latest(mdir)[0]
        assert 0 < step_at_pause < 4000
        jid2 = jm.control(jid, "resume")["job"]
        time.sleep(0.5)
        jm.control(jid2, "stop")
        assert jm.wait(jid2, 120) == "stopped"
        assert ckpt.latest(mdir)[0] >= step_at_pause
    finally:
        jm.shutdown()


# ---------------------------------------------------------------- inference
def test_prepare_reference_binarizes_and_centres():
    img = np.zeros((40, 40), np.uint8)
    img[5:35, 15:25] = 255
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="PNG")
    x = prepare_reference(b.getvalue()).reshape(28, 28)
    assert set(np.unique(x)) <= {0.0, np.float32(254 / 255)}
    assert x[:4].sum() == 0 and x[24:].sum() == 0 and x[:, :4].sum() == 0
    assert x.sum() > 0


def test_inference_service_cache(tmp_path):
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    svc = InferenceService(device="cpu")
    img = io.BytesIO()
    Image.fromarray(synthetic_mnist(1, seed=9).images[0].reshape(28, 28)).save(img, format="PNG")
    assert svc.predict(mdir, img.getvalue())["result"] == "fail"
    run_job(mdir, dict(SMALL, iter=10), device="cpu", backend="torch", data=_data())
    r1 = svc.predict(mdir, img.getvalue(), prep="mnist")
    r2 = svc.predict(mdir, img.getvalue(), prep="mnist")
    assert r1 == r2 and r1["result"] == "success"
    assert svc.misses == 1 and svc.hits >= 1
    many = svc.predict_many(mdir, [img.getvalue()] * 5)
    assert len(many) == 5 and all(m["result"] == "success" for m in many)
    # no per-model lock left behind after the load; a retired entry drops its
    # batchers (they referenced the entry: a cycle only the cyclic GC would free)
    assert svc._loading == {}
    ent = next(iter(svc._cache.values()))
    assert ent.batchers
    with svc._lock:
        ent.retire()
    assert ent.batchers == {} and ent.retired


def test_watchdog_kills_hung_worker(tmp_path, monkeypatch):
    s = _settings(tmp_path, "process")
    s.heartbeat_s = 4.0
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    monkeypatch.setenv("CSA_HANG_AT_STEP", "15")
    jm = JobManager(s, db, executor="process", ngpu=0)
    try:
        _prep_model(s, uid, "m")
        jid = jm.submit(uid, "m", "file", dict(SMALL, iter=100))
        assert jm.wait(jid, 240) == "failed"
        assert "heartbeat" in db.get_job(jid)["error"]
    finally:
        jm.shutdown()


def test_checkpoint_resume_across_flat_layouts():
    """Optimizer slots saved under the dense-last ("lowrank") layout re-map by name when
    the job resumes under the DSL-order layout of "allreduce"."""
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    cfg = parse_train_config(dict(SMALL, optimizer_name="AdagradOptimizer"))
    train, _ = _data()
    a = TrainEngine(cfg, train, strategy="lowrank")
    for _ in range(3):
        a.step()
    obj = ckpt.engine_state(a)
    b = TrainEngine(cfg, train, strategy="allreduce")
    assert a.model.state.offsets != b.model.state.offsets
    ckpt.restore_engine(b, obj)
    for n in a.model.state.shapes:
        torch.testing.assert_close(a.model.state.view(n, a.slots[0]), b.model.state.view(n, b.slots[0]))
        torch.testing.assert_close(a.model.state.view(n, a.flat), b.model.state.view(n, b.flat))


def test_auto_restart_from_checkpoint(tmp_path, monkeypatch):
    """SURVEY §5.3 recovery policy: a worker that fails after making progress is re-queued
    and resumes from its newest checkpoint (bounded); the fault fires once here."""
    s = _settings(tmp_path, "thread")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    monkeypatch.setenv("CSA_FAULT_AT_STEP", "25")
    monkeypatch.setenv("CSA_FAULT_ONCE", "1")
    jm = JobManager(s, db, executor="thread", ngpu=0)
    try:
        mdir = _prep_model(s, uid, "m")
        jid = jm.submit(uid, "m", "file", dict(SMALL, iter=30))
        t0 = time.time()
        while time.time() - t0 < 120:
            st = db.get_job(jid)["state"]
            if st in ("done", "failed"):
                break
            time.sleep(0.05)
        assert db.get_job(jid)["state"] == "done"
        assert "restart 1" in (db.get_job(jid)["error"] or "")  # recovered after restart 1
        assert json.load(open(os.path.join(mdir, STATUS)))["step"] == 30
    finally:
        jm.shutdown()


def test_fault_step_per_rank(monkeypatch, tmp_path):
    from cloud_server_amd.runtime.trainer import _fault_step
    monkeypatch.setenv("CSA_FAULT_AT_STEP", "1:7")
    assert _fault_step(1, str(tmp_path)) == 7 and _fault_step(0, str(tmp_path)) == -1
    monkeypatch.setenv("CSA_FAULT_AT_STEP", "9")
    assert _fault_step(0, str(tmp_path)) == 9 and _fault_step(3, str(tmp_path)) == 9


def test_tracing_ranges_wired(monkeypatch):
    """CSA_TRACE=1 turns on ROCTx ranges around steps / collectives / logs
    (the ROCTx library is part of the ROCm image; calls are no-ops without a profiler)."""
    from cloud_server_amd.utils import tracing
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    monkeypatch.setenv("CSA_TRACE", "1")
    monkeypatch.setattr(tracing, "_TRIED", False)
    monkeypatch.setattr(tracing, "_ROCTX", None)
    calls = []
    real = tracing.trace_range

    def spy(name):
        calls.append(name)
        return real(name)

    import cloud_server_amd.runtime.engine as E
    monkeypatch.setattr(E, "trace_range", spy)
    train, _ = _data()
    eng = TrainEngine(parse_train_config(SMALL), train, device="cpu")
    eng.step()
    eng.step()
    assert calls.count("csa.step") == 2
    assert tracing.enabled() == any(os.path.exists(os.path.join("/opt/rocm/lib", n))
                                    for n in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"))


def test_inference_micro_batcher_groups_concurrent_requests(tmp_path):
    """Requests queued while a batch runs are served by ONE forward (serve.inference)."""
    import threading
    from cloud_server_amd.serve.inference import _Batcher
    gate = threading.Event()
    sizes = []

    def fn(xs):
        gate.wait(5)
        sizes.append(len(xs))
        return xs[:, 0] * 2

    b = _Batcher(fn)
    futs = [b.submit(np.array([i], np.int64)) for i in range(10)]
    time.sleep(0.1)
    gate.set()
    assert [f.result(5) for f in futs] == [2 * i for i in range(10)]
    assert sum(sizes) == 10 and len(sizes) <= 2
    b.close()


def test_inference_service_async_path_cpu(tmp_path):
    import asyncio
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    run_job(mdir, dict(SMALL, iter=10), device="cpu", backend="torch", data=_data())
    svc = InferenceService(device="cpu")
    imgs = []
    for i in range(6):
        b = io.BytesIO()
        Image.fromarray(synthetic_mnist(6, seed=9).images[i].reshape(28, 28)).save(b, format="PNG")
        imgs.append(b.getvalue())

    async def go():
        return await asyncio.gather(*[svc.predict_async(mdir, im, prep="mnist") for im in imgs])
    out = asyncio.run(go())
    sync = [svc.predict(mdir, im, prep="mnist") for im in imgs]
    assert out == sync and all(o["result"] == "success" for o in out)
    assert svc.latency_ms()["n"] == 12
    svc.close()


# ---------------------------------------------------------------- single writer per model
def test_writer_lock_refuses_second_job_without_touching_status(tmp_path):
    """Two JobRuns on one model dir (e.g. two packed jobs in one GPU host): the second
    fails fast with LockHeld and leaves the first job's status/result files alone."""
    from cloud_server_amd.runtime.trainer import JobRun
    from cloud_server_amd.utils.locks import LockHeld
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    data = _data()
    a = JobRun(mdir, dict(SMALL, iter=20), device="cpu", backend="torch", data=data)
    st = open(os.path.join(mdir, STATUS)).read()
    with pytest.raises(LockHeld):
        JobRun(mdir, dict(SMALL, iter=20), device="cpu", backend="torch", data=data)
    assert open(os.path.join(mdir, STATUS)).read() == st
    while a.pending():
        a.before_step(); a.step(); a.after_step()
    assert a.finish()["state"] == "done"
    # released at finish: the next run of the model may write again
    b = JobRun(mdir, dict(SMALL, iter=30), device="cpu", backend="torch", data=data)
    b.fail(RuntimeError("x"))
    JobRun(mdir, dict(SMALL, iter=30), device="cpu", backend="torch", data=data)._unlock()


def test_one_job_per_model_conflict_and_supersede(tmp_path):
    """A second construct for a model whose job is queued/running is refused (JobConflict,
    HTTP 409); the first job's result.txt stays one clean run.  A paused job is
    superseded by a new construct, and resuming marks the old record 'resumed'."""
    from cloud_server_amd.runtime.jobs import JobConflict
    s = _settings(tmp_path, "thread")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor="thread", ngpu=0)
    try:
        mdir = _prep_model(s, uid, "m")
        cfg = dict(SMALL, iter=300, options=dict(SMALL["options"], log_every=20, ckpt_every=0))
        jid = jm.submit(uid, "m", "file", cfg)
        with pytest.raises(JobConflict):
            jm.submit(uid, "m", "file", dict(cfg, iter=7))
        assert json.load(open(os.path.join(mdir, "model.json")))["iter"] == 300     # not overwritten
        other = jm.submit(uid, "m2", "file", dict(SMALL, iter=5))                  # other models are free
        assert jm.wait(jid, 300) == "done" and jm.wait(other, 300) in ("done", "failed")
        lines = open(os.path.join(mdir, RESULT)).read().splitlines()
        steps = [int(l.split(",")[0].split(":")[1]) for l in lines if l.startswith("step:")]
        assert steps == list(range(0, 301, 20))          # (+ the reference's step == iter row)
        assert sum(l.startswith("final_accuracy:") for l in lines) == 1
        # paused -> a new construct supersedes it; resume of a paused job marks it resumed
        jid2 = jm.submit(uid, "m", "file", dict(cfg, iter=100000))
        t0 = time.time()
        while (db.get_job(jid2)["state"] != "running" or not os.path.exists(os.path.join(mdir, STATUS))
               or json.load(open(os.path.join(mdir, STATUS))).get("step", 0) <= 300) and time.time() - t0 < 120:
            time.sleep(0.05)
        jm.control(jid2, "pause")
        assert jm.wait(jid2, 120) == "paused"
        jid3 = jm.control(jid2, "resume")["job"]
        assert db.get_job(jid2)["state"] == "resumed"
        with pytest.raises(JobConflict):
            jm.submit(uid, "m", "file", cfg)
        jm.control(jid3, "pause")
        assert jm.wait(jid3, 120) == "paused"
        jid4 = jm.submit(uid, "m", "file", dict(cfg, iter=1))
        assert db.get_job(jid3)["state"] == "stopped" and "superseded" in db.get_job(jid3)["error"]
        assert jm.wait(jid4, 120) in ("done", "failed")
    finally:
        jm.shutdown()


def test_inference_reload_while_requests_in_flight(tmp_path):
    """A newer checkpoint loaded by one request closes the old entry's batchers; requests
    that resolved the old entry first must still complete (served by the old batcher or
    re-queued on the new entry), never hang behind the close sentinel."""
    import threading
    from cloud_server_amd.serve.inference import BatcherClosed, _Batcher
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    data = _data()
    run_job(mdir, dict(SMALL, iter=10), device="cpu", backend="torch", data=data)
    svc = InferenceService(device="cpu")
    b = io.BytesIO()
    Image.fromarray(synthetic_mnist(1, seed=9).images[0].reshape(28, 28)).save(b, format="PNG")
    img = b.getvalue()
    assert svc.predict(mdir, img, prep="mnist")["result"] == "success"
    stale = svc._entry(mdir)
    out, errs = [], []

    def client():
        try:
            for _ in range(20):
                out.append(svc.predict(mdir, img, prep="mnist")["result"])
        except Exception as exc:       # pragma: no cover - reported below
            errs.append(exc)
    ts = [threading.Thread(target=client) for _ in range(4)]
    for t in ts:
        t.start()
    run_job(mdir, dict(SMALL, iter=20), device="cpu", backend="torch", data=data)   # newer ckpt
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts) and not errs, errs
    assert out == ["success"] * 80
    assert stale.retired and all(bt.closed for bt in stale.batchers.values())
    with pytest.raises(BatcherClosed):                # a stale entry never grows a new batcher
        svc._batcher(stale, "reference")
    # submit after close fails fast; items queued before the close are still served
    bt = _Batcher(lambda xs: xs[:, 0])
    f = bt.submit(np.array([7], np.int64))
    bt.close()
    assert f.result(5) == 7
    with pytest.raises(BatcherClosed):
        bt.submit(np.array([1], np.int64))
    svc.close()


def test_scheduler_reserve_serving_slot():
    """The API process's serving slot: least-loaded placement avoids that GPU first and
    it never takes a GPU's last slot (runtime.jobs.JobManager.reserve_serving)."""
    for S in (NativeScheduler, PyScheduler):
        s = S(2, 2)
        assert s.reserve(-1000, 1) and s.load(1) == 1
        s.submit(1, 1); s.submit(2, 1); s.submit(3, 1); s.submit(4, 1)
        assert s.next() == (1, [0]) and s.next() == (2, [0]) and s.next() == (3, [1])
        assert s.next() is None and not s.reserve(-1000, 1) and not s.reserve(-1000, 7)
        assert s.release(-1000) == 1 and s.next() == (4, [1])


def test_job_manager_reserves_serving_slot(tmp_path):
    s = _settings(tmp_path, "thread")
    s.slots_per_gpu = 4
    jm = JobManager(s, Database(s.db_path), executor="thread", ngpu=2)
    try:
        assert jm.reserve_serving(1) == 1 and jm.sched.load(1) == 1 and jm.sched.load(0) == 0
        s.serve_slots = 4
        assert jm.reserve_serving(0) == 3            # the 4th would take the GPU's last slot
        assert jm.sched.load(0) == 3
        assert jm.release_serving() == 4 and jm.sched.load(0) == 0 and jm.sched.load(1) == 0
        # jobs already placed count — 2 serving slots on a GPU holding 2 jobs of 4
        s.serve_slots = 2
        assert jm.sched.reserve(7, 0) and jm.sched.reserve(8, 0)
        assert jm.reserve_serving(0) == 1 and jm.sched.load(0) == 3
        assert jm.release_serving() == 1 and jm.sched.load(0) == 2
    finally:
        jm.shutdown()


def test_capture_gc_guard_holds_across_overlapping_threads(monkeypatch):
    """two captures on different threads overlap — the collector stays off until
    the LAST one ends (a per-call save/restore re-enabled it under the other capture)."""
    import contextlib
    import gc
    import threading
    from cloud_server_amd.utils import graphs
    monkeypatch.setattr(torch.cuda, "graph", lambda *a, **k: contextlib.nullcontext())
    assert gc.isenabled() and graphs.active_captures() == 0
    a_in, b_in, a_out = threading.Event(), threading.Event(), threading.Event()
    seen = {}

    def first():
        with graphs.capture(object()):
            a_in.set()
            b_in.wait(10)
        a_out.set()

    def second():
        a_in.wait(10)
        with graphs.capture(object()):
            b_in.set()
            a_out.wait(10)
            seen["after_first_ended"] = gc.isenabled()

    ts = [threading.Thread(target=first), threading.Thread(target=second)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(20)
    assert seen["after_first_ended"] is False
    assert gc.isenabled() and graphs.active_captures() == 0


def test_job_manager_launches_8_gpu_dp_job(tmp_path):
    """an 8-GPU data-parallel job is placed on 8 distinct GPUs and launched
    as ONE torch.distributed.run with 8 local ranks over HIP_VISIBLE_DEVICES=0..7.  The
    captured launch line is then run for real (gloo, CPU): every rank sees WORLD_SIZE=8,
    LOCAL_WORLD_SIZE=8 and a distinct LOCAL_RANK (= its GPU under init_distributed)."""
    import subprocess
    import sys
    s = _settings(tmp_path, "process")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor="process", ngpu=8, slots_per_gpu=1)

    class _Q:
        def __init__(self):
            self.items = []

        def put(self, item):
            self.items.append(item)

    real, jm._req = jm._req, _Q()
    try:
        _prep_model(s, uid, "m8", n=40)
        jid = jm.submit(uid, "m8", "file", dict(SMALL, iter=4), ngpus=8)
        t0 = time.time()
        while not jm._req.items and time.time() - t0 < 30:
            time.sleep(0.05)
        kind, got, argv, env, mdir, log = jm._req.items[0]
        assert kind == "launch" and got == jid
        assert sorted(jm.running[jid]["gpus"]) == list(range(8))
        assert all(jm.sched.load(g) == 1 for g in range(8))
        assert env["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7"
        assert "--nproc-per-node=8" in argv and argv[1:3] == ["-m", "torch.distributed.run"]
        # run the launch line with a probe in place of the worker module's arguments
        i = argv.index("cloud_server_amd.runtime.worker")
        probe = tmp_path / "probe.py"
        probe.write_text(
            "import json, os\n"
            "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'HIP_VISIBLE_DEVICES']\n"
            f"open(os.path.join(r'{tmp_path}', 'probe_%s.json' % os.environ['RANK']), 'w').write("
            "json.dumps({k: os.environ.get(k) for k in keys}))\n")
        assert argv[i - 1] == "-m"          # torchrun runs the worker as a module
        cmd = argv[:i - 1] + [str(probe)]
        r = subprocess.run(cmd, env=dict(env, OMP_NUM_THREADS="1"), capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        seen = [json.load(open(tmp_path / f"probe_{k}.json")) for k in range(8)]
        assert sorted(int(d["LOCAL_RANK"]) for d in seen) == list(range(8))
        assert all(d["WORLD_SIZE"] == "8" and d["LOCAL_WORLD_SIZE"] == "8" for d in seen)
        assert all(d["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7" for d in seen)
    finally:
        jm._req = real
        jm.shutdown()


@pytest.mark.parametrize("strategy,variant", [("async_ps", "hf"), ("async_ps:flat", ""),
                                              ("allreduce", ""), ("allreduce:hf", "hf")])
def test_strategy_variant_parse(strategy, variant, monkeypatch):
    """``async_ps`` runs the ``:hf`` program by default (``async_ps:flat`` / CSA_APS_VARIANT
    keep the bucketed one); other strategies take the variant as written."""
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    monkeypatch.delenv("CSA_APS_VARIANT", raising=False)
    cfg = parse_train_config(dict(SAMPLE_CONFIG, options={"batch_size": 8}))
    eng = TrainEngine(cfg, synthetic_mnist(64, seed=0), device="cpu", strategy=strategy)
    assert eng.dp_variant == variant
    assert eng.sync.strategy == strategy.split(":")[0]
    monkeypatch.setenv("CSA_APS_VARIANT", "flat")
    if strategy == "async_ps":
        assert TrainEngine(cfg, synthetic_mnist(64, seed=0), device="cpu", strategy=strategy).dp_variant == ""


def test_strip_final_tail_keeps_one_increasing_run(tmp_path):
    """A resumed job's result.txt: the previous run's rows at or after the resume step and
    its final line are dropped before the new rows are appended (trainer._strip_final_tail),
    so the reference monitor still reads one increasing run of step lines."""
    from cloud_server_amd.runtime.trainer import _strip_final_tail
    p = tmp_path / "result.txt"
    rows = [f"step:{s},accuracy:0.5,duration:0.1\n" for s in range(0, 60, 10)]
    p.write_text("".join(rows) + "final_accuracy:0.9\n")
    _strip_final_tail(str(p), 40)
    assert p.read_text() == "".join(rows[:4])
    _strip_final_tail(str(p), 100)                     # nothing at/after 100, no final line
    assert p.read_text() == "".join(rows[:4])
    _strip_final_tail(str(tmp_path / "missing.txt"), 0)   # (no file: no-op)


def test_tail_timeout_knob_fires_once_per_model_dir(tmp_path, monkeypatch):
    """CSA_TAIL_TIMEOUT_AT_STEP arms the forced in-kernel timeout once per model dir (a
    marker file), so the automatic restart from the last checkpoint runs clean."""
    from cloud_server_amd.runtime.trainer import _tail_timeout_step
    monkeypatch.delenv("CSA_TAIL_TIMEOUT_AT_STEP", raising=False)
    assert _tail_timeout_step(str(tmp_path)) == -1
    monkeypatch.setenv("CSA_TAIL_TIMEOUT_AT_STEP", "45")
    assert _tail_timeout_step(str(tmp_path)) == 45
    assert os.path.exists(tmp_path / ".tail_timeout_fired")
    assert _tail_timeout_step(str(tmp_path)) == -1     # the restarted run is not re-armed

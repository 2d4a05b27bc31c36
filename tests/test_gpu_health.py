"""In-kernel timeouts are reported on every path.

The one-GPU program's pair-backward tail waits (bounded, 1 s) for the pair workgroups and,
on timeout, sets an error word and skips its work (conv / BatchNorm updates, statistic-slab
zeroing, next-batch staging).  ``HipProgram.arm_tail_timeout`` forces that timeout on the
next launch (the debug knob; ``CSA_TAIL_TIMEOUT_AT_STEP`` in a job).  The engine, the bench
and the job loop must all fail loudly on it, never train on."""
import json
import os
import time

import pytest
import torch

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    return parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3,
                                   options={"batch_size": 50}, **kw))


def test_forced_tail_timeout_is_reported_and_one_shot():
    eng = TrainEngine(_cfg(), synthetic_mnist(2000, seed=0), device="cuda:0", backend="hip")
    assert eng.backend == "hip", eng.fallback_reason
    assert eng.program.tail and eng.health_words(), "the one-GPU program has a pair-backward tail"
    for _ in range(6):                          # eager first step, then graph replays
        eng.step()
    eng.sync_device()
    eng.check_health()                          # healthy: no raise
    assert eng.program.tail_error() == 0
    before = eng.flat.clone()
    assert eng.program.arm_tail_timeout()
    t0 = time.perf_counter()
    eng.step()                                  # (a graph replay: the arm is stream-ordered)
    eng.sync_device()
    assert time.perf_counter() - t0 > 0.5       # the tail really waited out its bound
    assert eng.program.tail_error() == 1
    assert int(eng.program.tail_force.item()) == 0           # disarmed by the closing tail
    with pytest.raises(RuntimeError, match="in-kernel wait timed out"):
        eng.check_health()
    # the conv parameters were NOT updated by the timed-out tail (what would be silently
    # lost), while the dense layers were (their updates do not depend on the tail)
    conv = [n for n in eng.model.state.shapes if n.startswith(eng.program.units[0].layer.name)]
    assert conv and all(torch.equal(eng.model.state.view(n, eng.flat), eng.model.state.view(n, before))
                        for n in conv)
    # sticky: later healthy steps do not clear it
    eng.step()
    eng.sync_device()
    assert eng.program.tail_error() == 1


def test_job_with_tail_timeout_fails_then_restarts_from_checkpoint(tmp_path, monkeypatch):
    """The job loop reads the word: the job fails (status ``failed``, no checkpoint of the
    corrupted state), the manager re-queues it, and it resumes from the last good
    checkpoint and finishes."""
    from PIL import Image
    from cloud_server_amd.config import Settings
    from cloud_server_amd.runtime import checkpoint as ckpt
    from cloud_server_amd.runtime.jobs import JobManager
    from cloud_server_amd.runtime.trainer import STATUS
    from cloud_server_amd.store.db import Database
    monkeypatch.setenv("CSA_TAIL_TIMEOUT_AT_STEP", "45")
    s = Settings(storage_root=str(tmp_path / "s"), db_path=str(tmp_path / "db.sqlite3"),
                 executor="thread", train_backend="hip")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    mdir = s.model_dir(uid, "m")
    os.makedirs(os.path.join(mdir, "data"))
    ds = synthetic_mnist(300, seed=3)
    tags = {}
    for i in range(300):
        Image.fromarray(ds.images[i].reshape(28, 28)).save(os.path.join(mdir, "data", f"{i}.png"))
        tags[f"{i}.png"] = str(int(ds.labels[i]))
    json.dump(tags, open(os.path.join(mdir, "tag.json"), "w"))
    cfg = dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3, iter=100,
               options={"batch_size": 50, "log_every": 10, "ckpt_every": 20})
    jm = JobManager(s, db, executor="thread", ngpu=1)
    try:
        jid = jm.submit(uid, "m", "file", cfg)
        state = jm.wait(jid, 300)
        job = db.get_job(jid)
        assert state == "done", job
        err = job["error"] or ""
        # failed once on the timeout, restarted, recovered
        assert "restart 1" in err or "recovered after restart 1" in err, err
        assert os.path.exists(os.path.join(mdir, ".tail_timeout_fired"))
        assert json.load(open(os.path.join(mdir, STATUS)))["step"] == 100
        assert ckpt.latest(mdir)[0] == 100
        lines = open(os.path.join(mdir, "result.txt")).read().splitlines()
        steps = [int(ln.split(",")[0].split(":")[1]) for ln in lines if ln.startswith("step")]
        # the restart resumed from step 40 (the last checkpoint before the timeout at 45):
        # the failed run's rows from 40 on were dropped and re-logged once; the run is one
        # increasing sequence of step lines (0 .. 100: the reference's step == iter row),
        # then one final line
        assert steps == list(range(0, 101, 10)), steps
        assert sum(ln.startswith("final_accuracy:") for ln in lines) == 1
    finally:
        jm.shutdown()

"""Platform on the MI355X: a training job through the trainer (HIP kernels, HIP graph),
the job manager's process executor placing a worker on the GPU, the warm inference
cache on the device, and the reference's 99-image fixture end to end."""
import json
import os
import zipfile

import numpy as np
import pytest
import torch

from cloud_server_amd.config import Settings
from cloud_server_amd.data.datasets import load_user_data, synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG
from cloud_server_amd.runtime import checkpoint as ckpt
from cloud_server_amd.runtime.trainer import RESULT, read_train_results, run_job
from cloud_server_amd.serve.inference import InferenceService

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _cfg(iters, **opts):
    c = json.loads(json.dumps(SAMPLE_CONFIG))
    c.update(iter=iters, learning_rate=0.01, optimizer_name="AdamOptimizer")
    c["options"] = dict(log_every=100, ckpt_every=200, **opts)
    return c


def _close(*services) -> None:
    """Retire the services' cached models (their HIP graphs, batcher threads) NOW, in this
    thread: a later test's graph capture must never overlap their destruction."""
    import gc
    for s in services:
        s.close()
    gc.collect()
    torch.cuda.synchronize()


def test_gpu_job_hip_backend_and_inference(tmp_path):
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    ds = synthetic_mnist(6000, seed=0)
    out = run_job(mdir, _cfg(600), device="cuda:0", backend="hip", data=ds.split(0.9))
    assert out["backend"] == "hip" and out["state"] == "done" and out["step"] == 600
    res = read_train_results(os.path.join(mdir, RESULT), 600)
    assert [r["step"] for r in res["every_result"]] == [str(s) for s in range(0, 601, 100)]
    assert float(res["final_accuracy"]) > 0.9
    obj = ckpt.load(ckpt.latest(mdir)[1])
    assert obj["host_step"] == 600
    gpu = InferenceService(device="cuda:0")
    cpu = InferenceService(device="cpu")
    test = ds.split(0.9)[1]
    x = test.images[:256].astype(np.float32) / 255.0
    try:
        pg = gpu.predict_arrays(mdir, x)
        pc = cpu.predict_arrays(mdir, x)
        assert (pg == pc).mean() > 0.99
        assert (pg == test.labels[:256]).mean() > 0.9
    finally:
        _close(gpu, cpu)


def test_gpu_job_on_reference_fixture(tmp_path):
    """The reference's 99 labelled digit JPEGs (test-data/) as a user dataset."""
    mdir = str(tmp_path / "m")
    os.makedirs(os.path.join(mdir, "data"))
    with zipfile.ZipFile(os.path.join(FIX, "test-pics.zip")) as z:
        z.extractall(os.path.join(mdir, "data"))
    with open(os.path.join(FIX, "tag.json"), "rb") as f, open(os.path.join(mdir, "tag.json"), "wb") as g:
        g.write(f.read())
    out = run_job(mdir, _cfg(300), datatype="file", device="cuda:0", backend="hip")
    assert out["state"] == "done" and out["backend"] == "hip"
    ds = load_user_data(os.path.join(mdir, "data"), os.path.join(mdir, "tag.json"))
    svc = InferenceService(device="cuda:0")
    try:
        pred = svc.predict_arrays(mdir, ds.images[:79].astype(np.float32) / 255.0)
        assert (pred == ds.labels[:79]).mean() > 0.9        # fits its training split
    finally:
        _close(svc)


def test_job_manager_process_executor_on_gpu(tmp_path):
    from cloud_server_amd.runtime.jobs import JobManager
    from cloud_server_amd.store.db import Database
    from PIL import Image
    s = Settings(storage_root=str(tmp_path / "s"), db_path=str(tmp_path / "db.sqlite3"),
                 executor="process", train_backend="hip")
    db = Database(s.db_path)
    uid = db.create_user("u", "pw-12345678")
    jm = JobManager(s, db, executor="process", ngpu=1)
    try:
        mdir = s.model_dir(uid, "m")
        os.makedirs(os.path.join(mdir, "data"))
        ds = synthetic_mnist(500, seed=3)
        tags = {}
        for i in range(500):
            Image.fromarray(ds.images[i].reshape(28, 28)).save(os.path.join(mdir, "data", f"{i}.png"))
            tags[f"{i}.png"] = str(int(ds.labels[i]))
        json.dump(tags, open(os.path.join(mdir, "tag.json"), "w"))
        os.makedirs(s.model_dir(uid, "m2"))
        os.symlink(os.path.join(mdir, "data"), os.path.join(s.model_dir(uid, "m2"), "data"))
        json.dump(tags, open(os.path.join(s.model_dir(uid, "m2"), "tag.json"), "w"))
        # two jobs on one GPU: packed into that GPU's host process (settings.pack_jobs)
        jids = [jm.submit(uid, "m", "file", _cfg(200)), jm.submit(uid, "m2", "file", _cfg(300))]
        hlog = os.path.join(s.storage_root, "gpu_hosts", "gpu0", "host.log")
        for jid in jids:
            state = jm.wait(jid, 400)
            log = open(hlog).read() if os.path.exists(hlog) else ""
            assert state == "done", log[-3000:]
            st = jm.status(jid)
            assert st["gpu"] == "0" and st["progress"]["backend"] == "hip"
        assert jm.status(jids[1])["progress"]["step"] == 300
    finally:
        jm.shutdown()


def _ring_losses(e):
    from cloud_server_amd.runtime.engine import RING
    torch.cuda.synchronize()
    pos = torch.tensor([i % RING for i in range(e.host_step)], device=e.ring_loss.device)
    return e.ring_loss.index_select(0, pos).double().cpu()


def test_packed_hip_jobs_match_solo():
    """K jobs as branches of one graph (runtime.multijob) train exactly like solo jobs
    (atomic split-K sums: fp32 reassociation tolerance)."""
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    from cloud_server_amd.runtime.multijob import PackedJobs

    def eng(seed, packed=False):
        c = _cfg(100, seed=seed)
        c.update(optimizer_name="AdagradOptimizer", learning_rate=1e-3)
        return TrainEngine(parse_train_config(c), synthetic_mnist(2000, seed=seed), device="cuda:0", backend="hip",
                           packed=packed)

    solo = [eng(s) for s in (1, 2, 3)]
    for e in solo:
        for _ in range(20):
            e.step()
    # the packed launch profile (two pooled rows per conv-pair workgroup, 128-column fused
    # dense blocks) trains like the solo profile
    packed = [eng(s, packed=True) for s in (1, 2, 3)]
    assert all(e.backend == "hip" for e in solo + packed)
    assert all(e.program.packed for e in packed) and not any(e.program.packed for e in solo)
    pack = PackedJobs(packed)
    for _ in range(20):
        pack.step()
    pack.sync_device()
    for a, b in zip(solo, packed):
        # a handful of the 2.3 M parameters land ~1e-4 apart: split-K / statistic atomics
        # sum in a different order in the two runs (seen on 5 head weights, once)
        torch.testing.assert_close(b.flat, a.flat, rtol=1e-3, atol=5e-4)
        # this config's loss (~8-24) amplifies the reassociation noise: two SOLO runs of the
        # same seed drift apart by ~1.5% in the last step's loss (measured, round 3), so the
        # early steps are pinned tightly and the 20-step mean to the solo-vs-solo noise
        la, lb = _ring_losses(a), _ring_losses(b)
        torch.testing.assert_close(lb[:8], la[:8], rtol=1e-4, atol=1e-4)
        assert abs(float(la.mean() - lb.mean())) < 1e-2 * float(la.mean())


def test_production_job_loop_matches_bench_throughput(tmp_path):
    """The trainer loop (logging every 100 steps from the device metric ring, time-based
    async checkpoints, control polling) keeps >= 90% of the bare engine's step rate."""
    import time
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    c = json.loads(json.dumps(SAMPLE_CONFIG))
    c.update(iter=20000, learning_rate=1e-4, optimizer_name="AdagradOptimizer")
    c["options"] = dict(batch_size=50, ckpt_secs=1)        # several async checkpoints in the run
    ds = synthetic_mnist(20000, seed=0)
    e = TrainEngine(parse_train_config(c), ds, device="cuda:0", backend="hip")
    for _ in range(200):
        e.step()
    e.sync_device()
    t0 = time.perf_counter()
    for _ in range(4000):
        e.step()
    e.sync_device()
    bench = 50 * 4000 / (time.perf_counter() - t0)
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    t0 = time.perf_counter()
    out = run_job(mdir, c, device="cuda:0", backend="hip", data=ds.split(0.95))
    wall = time.perf_counter() - t0
    assert out["state"] == "done" and out["backend"] == "hip"
    rows = [json.loads(l) for l in open(os.path.join(mdir, "metrics.jsonl"))]
    sps = sorted(r["samples_per_s"] for r in rows[5:])
    median = sps[len(sps) // 2]
    print(f"bench {bench:.0f} samples/s, job loop median {median:.0f} samples/s, "
          f"{len(rows)} log lines, wall {wall:.1f}s, checkpoints kept {len(ckpt.list_checkpoints(mdir))}")
    assert median >= 0.9 * bench, (median, bench)


def test_node_status_reports_gpus_on_device():
    """GET /runtime/kubernetes/ analogue on a real node: amdsmi sees the MI355X and the
    report carries its VRAM and (where the driver exposes them) xGMI link fields."""
    from cloud_server_amd.runtime.devices import node_status
    st = node_status([])
    assert st["Capacity"]["amd.com/gpu"] != "0", st["Conditions"]
    g = st["GPUs"][0]
    assert "vram" in g or "asic" in g, sorted(g)
    assert isinstance(st["Topology"], list)
    print("gpu0 fields:", sorted(g))


def test_packed_run_steps_equal_single_packed_steps(monkeypatch):
    """PackedJobs.run_steps(n) (8-step multi-job graphs, groups never crossing a half of a
    job's row table: stream_chunk 12 forces half switches inside the run) == n single
    packed steps: same host/device step, cursor, per-step batches and weights (gpu_host's
    default path).  The sample config's saturated logits amplify fp32 atomic-order noise
    chaotically: two IDENTICAL single-step runs already disagree by O(1) in the loss after
    ~10 steps (scripts/diag_group.py), so batches and numerics are compared over the first
    groups, at a small SGD rate, and the counters over the whole run."""
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    from cloud_server_amd.runtime.multijob import PackedJobs

    # 8-step groups: they fit the 12-step row-table chunks (the default 32 would not group)
    monkeypatch.setenv("CSA_GRAPH_STEPS", "8")

    def engs():
        out = []
        for seed in (1, 2):
            c = _cfg(100, seed=seed)
            c.update(optimizer_name="GradientDescentOptimizer", learning_rate=1e-4)
            out.append(TrainEngine(parse_train_config(c), synthetic_mnist(2000, seed=seed), device="cuda:0",
                                   backend="hip", stream_chunk=12))
        return out
    a, b = PackedJobs(engs()), PackedJobs(engs())
    a.step(); b.step()
    a.run_steps(40)
    for _ in range(40):
        b.step()
    a.sync_device()
    assert a.graph_k is not None and a.host_step == b.host_step == 41
    for x, y in zip(a.engines, b.engines):
        assert x.host_step == y.host_step == 41 and int(x.dstep.item()) == int(y.dstep.item()) == 41
        assert torch.equal(x.stream.cursor, y.stream.cursor)
        # the same batch every step: per-step loss and #correct agree while the two runs'
        # weights are still within fp32 noise of each other
        torch.testing.assert_close(x.ring_loss[:9], y.ring_loss[:9], rtol=1e-4, atol=1e-5)
        assert (x.ring_correct[:9] - y.ring_correct[:9]).abs().max().item() <= 1


def test_packed_readmission_recaptures_without_rewarming():
    """Admitting a job into a running pack re-captures the graph without re-running the
    hosted jobs' warm-up (their weights / step counters are untouched by the re-pack) and
    the stall is one capture; the hosted job then continues exactly as a lone run."""
    import time
    from cloud_server_amd.models.dsl import parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    from cloud_server_amd.runtime.multijob import PackedJobs

    def eng(seed):
        c = _cfg(100, seed=seed)
        c.update(optimizer_name="AdagradOptimizer", learning_rate=1e-3)
        return TrainEngine(parse_train_config(c), synthetic_mnist(2000, seed=seed), device="cuda:0", backend="hip")
    old, solo = eng(1), eng(1)
    p1 = PackedJobs([old])
    for _ in range(10):
        p1.step(); solo.step()
    p1.sync_device()
    before = old.flat.clone()
    new = eng(2)
    p2 = PackedJobs([old, new])
    t0 = time.perf_counter()
    p2._capture()
    torch.cuda.synchronize()
    stall = time.perf_counter() - t0
    assert torch.equal(old.flat, before) and int(old.dstep.item()) == 10     # nothing ran
    print(f"re-pack stall with one new job: {stall * 1e3:.1f} ms")
    for _ in range(10):
        p2.step(); solo.step()
    p2.sync_device()
    torch.testing.assert_close(old.flat, solo.flat, rtol=1e-3, atol=5e-4)

"""bench.py driver contract on CPU: the N > 1 path under torch.distributed.run (gloo,
world 2, 127.0.0.1 rendezvous) prints ONE JSON line from rank 0 with the whole-job value,
n_gpus, the weak-scaling config and the start-up strategy timings."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_world2_cpu_one_json_line():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["metric"] == "train_samples_per_s" and d["n_gpus"] == 2 and d["steps"] == 2
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["global_batch"] == 100 and d["config"]["per_gpu_batch"] == 50
    assert d["config"]["parallelism"].startswith("dp2")
    assert d["config"]["collectives"] == "gloo"
    assert set(d["config"]["strategy_tuning_ms_per_step"]) == {"lowrank", "allreduce", "ps"}
    assert d["value"] > 0 and d["ms_per_step"] > 0


class _FakeGraph:
    """Stands in for a captured HIP graph on CPU: a replay counts itself and perturbs the
    parameters the way a real replay would (so a missing restore is visible)."""
    log = []

    def __init__(self, eng=None, k=0):
        self.eng, self.k, self.replays = eng, k, 0

    def replay(self):
        self.replays += 1
        _FakeGraph.log.append(self.k)
        if self.eng is not None:
            self.eng.flat.add_(1.0)
            self.eng.dstep.add_(self.k)


def test_run_steps_warm_replay_and_remainder_graphs(monkeypatch):
    """bench.py contract (VERDICT r3 'next' #2): prepare_group_graph captures the 8/4/2-step
    graphs and replays each ONCE with the model state restored, so no graph's first launch
    lands in the timed loop; run_steps(n) then covers n mod 8 with the 4/2-step graphs and
    runs at most one single-step replay."""
    import contextlib
    import torch
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.runtime import engine as E

    cfg = parse_train_config(dict(SAMPLE_CONFIG, options={"batch_size": 8}))
    eng = E.TrainEngine(cfg, synthetic_mnist(64, seed=0), device="cpu")
    made = []

    class Graph(_FakeGraph):
        def __init__(self):
            super().__init__(eng, 0)
            made.append(self)

    @contextlib.contextmanager
    def fake_capture(g):
        n0 = calls[0]
        yield
        g.k = calls[0] - n0            # steps recorded into this graph

    calls = [0]
    monkeypatch.setattr(eng.program, "run", lambda: calls.__setitem__(0, calls[0] + 1))
    monkeypatch.setattr(E, "capture", fake_capture)
    monkeypatch.setattr(torch.cuda, "CUDAGraph", Graph)
    monkeypatch.setattr(eng, "group_steps", lambda: 8)
    eng.use_graph = True
    eng.graph = _FakeGraph(eng, 1)           # the single-step graph (already warm)
    before = (eng.flat.clone(), eng.dstep.clone(), eng.stream.cursor.clone())
    _FakeGraph.log = []
    eng.prepare_group_graph()
    assert sorted(eng.graphs_k) == [2, 4, 8] and [g.k for g in made] == [8, 4, 2]
    assert all(g.replays == 1 for g in made)                     # warm replay of every size
    assert torch.equal(eng.flat, before[0]) and torch.equal(eng.dstep, before[1])
    assert torch.equal(eng.stream.cursor, before[2])             # state restored
    _FakeGraph.log = []
    eng.run_steps(23)                                            # 8 + 8 + 4 + 2 + 1
    assert _FakeGraph.log == [8, 8, 4, 2, 1]
    assert eng.host_step == 23
    _FakeGraph.log = []
    eng.run_steps(6)
    assert _FakeGraph.log == [4, 2]


def test_bench_gpus2_without_torchrun_launches_two_ranks():
    """``python bench.py --gpus 2`` (no outer torchrun) runs two ranks —
    bench.py starts torch.distributed.run as a child and relays rank 0's JSON line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--strategy", "allreduce"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 100
    assert d["config"]["parallelism"].startswith("dp2")


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1",
           "--warmup", "0"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr and not out.stdout.strip()


import pytest  # noqa: E402


@pytest.mark.gpu
def test_bench_gpus2_rehearsal_on_one_gpu():
    """The driver's N-GPU bench path on the GPU box: ``bench.py --gpus 2`` (it starts
    torch.distributed.run itself) with both ranks on cuda:0 over gloo and the xGMI
    collectives (CSA_DIST_SHARED_GPU=1): strategy tuner, HIP programs, timed loop, one JSON
    line marked as a rehearsal."""
    env = dict(os.environ, CSA_DIST_SHARED_GPU="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                          "--warmup", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    c = d["config"]
    assert d["n_gpus"] == 2 and c["global_batch"] == 100 and c["backend"] == "hip"
    assert "rehearsal" in c and c["parallelism"].startswith("dp2")
    assert c["collectives"] and all(v == "xgmi" for v in c["collectives"].values()), c["collectives"]
    assert {"allreduce", "allreduce:hf", "ps", "ps:hf"} <= set(c["strategy_tuning_ms_per_step"])

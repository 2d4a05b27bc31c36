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
    assert set(d["config"]["strategy_tuning_ms_per_step"]) == {"lowrank", "allreduce"}
    assert d["value"] > 0 and d["ms_per_step"] > 0

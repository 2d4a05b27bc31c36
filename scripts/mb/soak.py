"""Soak run: N steps of the one-GPU program (32-step graphs, the production loop's shape)
with the in-kernel health words checked every ``chunk`` steps; prints one line per chunk
(steps, ms/step, loss, batch accuracy) and fails loudly on a timed-out wait."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bench import _sample_cfg  # noqa: E402
from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.runtime.engine import TrainEngine  # noqa: E402


class _A:
    optimizer = "AdagradOptimizer"
    batch = 50


def main():
    total = int(os.environ.get("SOAK_STEPS", "1000000"))
    chunk = int(os.environ.get("SOAK_CHUNK", "100000"))
    eng = TrainEngine(_sample_cfg(_A), synthetic_mnist(60000, seed=0), device="cuda:0", backend="hip", use_graph=True)
    eng.step()
    eng.prepare_group_graph()
    done = 1
    while done < total:
        n = min(chunk, total - done)
        t0 = time.perf_counter()
        eng.run_steps(n)
        eng.sync_device()
        dt = time.perf_counter() - t0
        done += n
        eng.check_health()
        m = eng.metrics_since(eng.host_step - 100)
        print(f"steps {done} ms/step {dt * 1e3 / n:.5f} loss {m['loss']:.4f} acc {m['accuracy']:.3f} "
              f"tail_err {eng.program.tail_error()}", flush=True)


if __name__ == "__main__":
    main()

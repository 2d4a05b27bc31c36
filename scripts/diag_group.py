"""Grouped (multi-step graph) vs single-step replays: per-step loss difference, packed and
solo, Adagrad.  A batch mismatch shows as a large loss jump at one step; fp32 atomic
reordering as ~1e-6 noise."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine
from cloud_server_amd.runtime.multijob import PackedJobs

def eng(seed, chunk):
    c = dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3, options={"batch_size": 50})
    cfg = parse_train_config(c); cfg.seed = seed
    return TrainEngine(cfg, synthetic_mnist(2000, seed=seed), device="cuda:0", backend="hip", stream_chunk=chunk)

def report(tag, xs, ys, n):
    for i, (x, y) in enumerate(zip(xs, ys)):
        dl = (x.ring_loss[:n] - y.ring_loss[:n]).abs()
        dc = (x.ring_correct[:n] - y.ring_correct[:n]).abs()
        print(f"{tag} job{i}: max dloss {dl.max().item():.3e} at step {int(dl.argmax())}, "
              f"first step with dloss>1e-4: {int((dl > 1e-4).nonzero()[0]) if (dl > 1e-4).any() else -1}, "
              f"dcorrect max {int(dc.max())}, dflat {(x.flat - y.flat).abs().max().item():.3e}")

for chunk in (12, 512):
    a, b = PackedJobs([eng(1, chunk), eng(2, chunk)]), PackedJobs([eng(1, chunk), eng(2, chunk)])
    a.step(); b.step(); a.run_steps(40)
    for _ in range(40): b.step()
    torch.cuda.synchronize(); report(f"packed chunk={chunk}", a.engines, b.engines, 41)
    # repeat single vs single (pure noise floor)
    c = PackedJobs([eng(1, chunk), eng(2, chunk)])
    for _ in range(41): c.step()
    torch.cuda.synchronize(); report(f"packed-single vs packed-single chunk={chunk}", c.engines, b.engines, 41)
    s1, s2 = eng(1, chunk), eng(1, chunk)
    s1.step(); s1.prepare_group_graph(); s1.run_steps(40)
    for _ in range(41): s2.step()
    torch.cuda.synchronize(); report(f"solo chunk={chunk}", [s1], [s2], 41)

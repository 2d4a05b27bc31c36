"""Per-step loss agreement of runs that must see identical batches (GD, small lr, so the
weights stay within fp32 noise): solo step() vs solo step(), solo run_steps vs step(),
packed single vs packed single, packed grouped vs packed single.  A mismatch of O(1) in
the loss of one step means that step trained on a different batch."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine
from cloud_server_amd.runtime.multijob import PackedJobs

STAGE = os.environ.get("CSA_STAGE_BATCH", "1")

def eng(seed, chunk):
    c = dict(SAMPLE_CONFIG, optimizer_name="GradientDescentOptimizer", learning_rate=1e-3, options={"batch_size": 50})
    cfg = parse_train_config(c); cfg.seed = seed
    return TrainEngine(cfg, synthetic_mnist(2000, seed=seed), device="cuda:0", backend="hip", stream_chunk=chunk)

def report(tag, xs, ys, n=41):
    for i, (x, y) in enumerate(zip(xs, ys)):
        dl = (x.ring_loss[:n] - y.ring_loss[:n]).abs()
        bad = (dl > 1e-3).nonzero().flatten().tolist()
        print(f"[stage={STAGE}] {tag} job{i}: bad steps {bad[:12]}{'...' if len(bad) > 12 else ''} "
              f"max dloss {dl.max().item():.2e}; dflat {(x.flat - y.flat).abs().max().item():.2e}", flush=True)

for chunk in (12, 512):
    s1, s2 = eng(1, chunk), eng(1, chunk)
    for _ in range(41): s1.step(); s2.step()
    torch.cuda.synchronize(); report(f"solo step vs step chunk={chunk}", [s1], [s2])
    s3 = eng(1, chunk)
    s3.step(); s3.prepare_group_graph(); s3.run_steps(40)
    torch.cuda.synchronize(); report(f"solo run_steps vs step chunk={chunk}", [s3], [s2])
    e1 = eng(1, chunk); e1.use_graph = False
    for _ in range(41): e1.step()
    torch.cuda.synchronize(); report(f"solo eager vs graph step chunk={chunk}", [e1], [s2])
    b = PackedJobs([eng(1, chunk), eng(2, chunk)])
    for _ in range(41): b.step()
    torch.cuda.synchronize(); report(f"packed single vs solo step chunk={chunk}", b.engines[:1], [s2])
    a = PackedJobs([eng(1, chunk), eng(2, chunk)])
    a.step(); a.run_steps(40)
    torch.cuda.synchronize(); report(f"packed grouped vs packed single chunk={chunk}", a.engines, b.engines)

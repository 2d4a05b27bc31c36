"""Timing probe (GPU): one captured step per graph vs k steps per graph (same program)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine

cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-4, options={"batch_size": 50}))
eng = TrainEngine(cfg, synthetic_mnist(60000), device="cuda", backend="hip", use_graph=True)
for _ in range(20):
    eng.step()
torch.cuda.synchronize()
for k in (1, 2, 4, 8):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(k):
            eng.program.run()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    n = 2000 // k
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    print(f"k={k}: {s.elapsed_time(e) * 1e3 / (n * k):.2f} us/step")

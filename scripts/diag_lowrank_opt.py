import os, socket, sys, torch, torch.distributed as dist
sys.path.insert(0, os.getcwd())
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.parallel.dist import DistContext
from cloud_server_amd.runtime.engine import TrainEngine
class D(DistContext):
    @property
    def enabled(self): return True
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CSA_XGMI="0")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for opt, lr in [("AdagradOptimizer", 1e-2), ("AdagradOptimizer", 1e-4), ("AdamOptimizer", 1e-3), ("GradientDescentOptimizer", 1e-2)]:
  for strat in ["lowrank", "allreduce"]:
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name=opt, learning_rate=lr))
    ds = synthetic_mnist(2000, seed=0)
    ctx = D(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy=strat)
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    res = []
    for k in range(20):
        a.step(); b.step()
        if k in (0, 1, 19):
            torch.cuda.synchronize()
            worst = max(((a.model.state.view(n, a.flat) - b.model.state.view(n, b.flat)).abs().max().item(), n) for n in a.model.state.shapes)
            res.append((k, round(worst[0], 6), worst[1]))
    print(opt, lr, strat, res, flush=True)
dist.destroy_process_group()

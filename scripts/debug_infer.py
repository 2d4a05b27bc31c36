"""Compare the HIP predict forward with the eager model layer by layer (GPU debug aid)."""
import json
import numpy as np
import torch
from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine
from cloud_server_amd.serve.hip_infer import _Bucket

c = json.loads(json.dumps(SAMPLE_CONFIG))
c.update(iter=100, learning_rate=0.01, optimizer_name="AdamOptimizer")
cfg = parse_train_config(c)
ds = synthetic_mnist(2000, seed=0)
eng = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
for _ in range(int(__import__("os").environ.get("STEPS", "50"))):
    eng.step()
eng.sync_device()
state = eng.model.export_state()
for k in state:
    if k.startswith("buffers."):
        print(k, state[k][:4])
B = 16
bk = _Bucket(cfg, state, B, torch.device("cuda:0"), "mnist")
x = ds.images[:B]
pred = bk.run(x)
net = bk.eng.model
xf = torch.from_numpy(x.astype(np.float32) / 255.0).cuda()
with torch.no_grad():
    h = xf.reshape(B, 28, 28, 1)
    outs = []
    for lp in net.plan.layers:
        h = net._layer(lp, h, False)
        outs.append((lp.spec.__class__.__name__, h))
    logits = h.reshape(B, -1) @ net.p("head.weight") + net.p("head.bias")
prog = bk.eng.program
for i, u in enumerate(prog.units):
    print("unit", i, u.kind, tuple(u.y.shape))
for name, t in outs:
    print(name, tuple(t.shape), float(t.abs().mean()))
# pair output = post-pool conv2 (layer index 3?)
for i, u in enumerate(prog.units):
    cands = [t for n, t in outs if t.numel() == u.y.numel()]
    for t in cands:
        d = (u.y.reshape(-1) - t.reshape(-1)).abs().max().item()
        print(f"unit {i} vs eager tensor of same size: maxdiff {d:.3e} (scale {t.abs().max().item():.3e})")
print("logits maxdiff", (bk.logits - logits).abs().max().item(), "scale", logits.abs().max().item())
print("pred", pred, "eager", logits.argmax(1).cpu().numpy())
u2 = prog.units[2]
tf = u2.in_tf
print("eval_slab mean diff", (tf.eval_slab[0, 0] - net.bn3_mean).abs().max().item(),
      "sumsq diff", (tf.eval_slab[0, 1] - (net.bn3_var + net.bn3_mean ** 2)).abs().max().item())
act_t = [t for n, t in outs if n == "ActSpec"][0]
print("xt vs eager act output", (u2.xt.reshape(-1) - act_t.reshape(-1)).abs().max().item())
norm_t = [t for n, t in outs if n == "NormSpec"][0]
# recompute the BN apply with the batch stats of this batch (what the training forward does)
pool_t = [t for n, t in outs if n == "PoolSpec"][0]
m = pool_t.mean(dim=(0, 1, 2)); v = pool_t.var(dim=(0, 1, 2), unbiased=False)
sc, of = net.p("norm3.scale") if "norm3.scale" in net.state.shapes else None, None
print([k for k in net.state.shapes])

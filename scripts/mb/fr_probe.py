import os, json, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", TORCH_NCCL_TRACE_BUFFER_SIZE="256")
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
t = torch.ones(4, device=dev)
dist.all_reduce(t)
from torch._C._distributed_c10d import _dump_nccl_trace_json
d = json.loads(_dump_nccl_trace_json(includeCollectives=True, onlyActive=True))
print("active keys", list(d.keys()), [ {k: e.get(k) for k in ("process_group", "state", "profiling_name")} for e in d.get("entries", [])][:3])
d = json.loads(_dump_nccl_trace_json(includeCollectives=True, onlyActive=False))
print("all", [ {k: e.get(k) for k in ("process_group", "state")} for e in d.get("entries", [])][:3])
print("name", dist.distributed_c10d._get_process_group_name(dist.distributed_c10d._get_default_group()))
o = dist.ProcessGroupNCCL.Options(); o.is_high_priority_stream = True
g = dist.new_group(backend="nccl", device_id=dev, pg_options=o)
dist.all_reduce(t, group=g); torch.cuda.synchronize()
print("hp group ok", t.tolist())
dist.destroy_process_group()

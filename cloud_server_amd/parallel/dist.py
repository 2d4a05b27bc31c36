"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL/xGMI.

Replaces the reference's TF ``ClusterSpec``/``tf.train.Server`` gRPC cluster
(construct_distribute.py:344-349) and the ``--ps_hosts/--worker_hosts/--job_name/
--task_index`` flags (:37-43).  Ranks come from the standard env:// variables that
``torch.distributed.run`` (or the job manager's launcher, ``runtime.jobs``) sets:
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT.

On ROCm the ``nccl`` backend IS RCCL; CPU tests use ``gloo`` with the same code.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def enabled(self) -> bool:
        return self.world > 1

    @property
    def is_chief(self) -> bool:
        return self.rank == 0   # reference: is_chief = task_index == 0 (:385)


def rccl_env_defaults() -> None:
    """Environment an RCCL process group of this package is created with (set before
    ``init_process_group``; explicit user settings win):

    * ``TORCH_NCCL_CUDA_EVENT_CACHE=0`` — RCCL collectives are captured into the step's HIP
      graphs; with the process-wide event cache a work's end event can be one last
      recorded inside a capture, which the watchdog may not query (hipErrorCapturedEvent);
    * ``NCCL_RUNTIME_CONNECT=0`` — every connection set up when a communicator is created,
      so the first collective of the dedicated capture group
      (``GradSync._setup_capture_group``) may be one inside a capture;
    * ``TORCH_NCCL_TRACE_BUFFER_SIZE`` — the flight recorder, whose active list tells when
      the watchdog has retired that group's one eager collective (``utils.graphs.wait_retired``);
    * ``TORCH_NCCL_BLOCKING_WAIT=1`` — no watchdog thread at all.  The separate capture
      group, the streams outside torch's pool and the retirement wait made the watchdog's
      hipErrorCapturedEvent abort rare, but it still hit one world-1 ``allreduce`` run in the
      round-5 closing check (``profiles/r5_notes.md``).  Without the thread nothing queries an
      event of a capturing stream.  Measured on this torch (2.10.0+rocm7.0, RCCL 2.26.6): with
      blocking wait the process has no ``pt_nccl_watchdg`` / ``pt_nccl_heartbt`` thread, without
      it both run (``tests/test_gpu_rccl_threads.py``, ``profiles/r6_notes.md``).  Eager collectives (set-up, agreement flags, log points)
      then block the host until they finish, and a hung one raises after the group timeout
      instead of being aborted by the watchdog.  Measured: the DP GPU tests and 3 x 4 world-1
      DP benches at unchanged ms/step (``scripts/gpu_r5bw.sh``)."""
    os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    os.environ.setdefault("NCCL_RUNTIME_CONNECT", "0")
    os.environ.setdefault("TORCH_NCCL_TRACE_BUFFER_SIZE", "256")


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_distributed(device_type: str = "auto", timeout_s: float = 300.0) -> DistContext:
    """Initialise from env. ``device_type``: 'cuda' (RCCL), 'cpu' (gloo) or 'auto'."""
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type == "auto":
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    # CSA_DIST_SHARED_GPU=1: a REHEARSAL of the N-rank GPU path on a box with fewer GPUs —
    # every rank on cuda:0, a gloo process group (RCCL refuses two ranks on one device),
    # every collective on the xGMI peer-buffer kernels (CSA_XGMI=1), the blocks of a call
    # capped so the ranks' kernels stay co-resident (the device tests' set-up)
    rehearse = device_type == "cuda" and world > 1 and os.environ.get("CSA_DIST_SHARED_GPU") == "1"
    if rehearse:
        from .xgmi import shared_gpu_block_cap
        os.environ["CSA_XGMI"] = "1"
        os.environ.setdefault("CSA_XGMI_BLOCKS", str(shared_gpu_block_cap(world)))
        os.environ.setdefault("LOCAL_WORLD_SIZE", str(world))
        local_rank = 0
        torch.cuda.set_device(0)
        device = torch.device("cuda", 0)
        backend = "gloo"
    elif device_type == "cuda":
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        backend = "nccl"
    else:
        device = torch.device("cpu")
        backend = "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
            rccl_env_defaults()
        dist.init_process_group(**kw)
    # (rehearsal: the GPU code paths of an RCCL job — xGMI collectives, HIP programs — on
    # the gloo group, as the multi-process device tests run them)
    label = "nccl" if rehearse else backend
    return DistContext(rank, world, local_rank, label if world > 1 else "none", device)


def barrier(ctx: DistContext) -> None:
    if ctx.enabled:
        if ctx.backend == "nccl" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[ctx.local_rank])
        else:
            dist.barrier()


def all_reduce_max(ctx: DistContext, value: float) -> float:
    if not ctx.enabled:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def ranks_share_gpu(ctx: DistContext, device: torch.device) -> bool:
    """True when another rank of this job drives the same physical GPU (the one-GPU
    multi-process tests; a node runs one rank per GPU).  Ranks compare PCI locations, so a
    launcher that narrows each rank's visible devices is not mistaken for sharing.  Called
    by every rank at engine construction (one small all-gather)."""
    if not ctx.enabled or device.type != "cuda" or not dist.is_initialized():
        return False
    p = torch.cuda.get_device_properties(device)
    me = (int(getattr(p, "pci_domain_id", 0)), int(getattr(p, "pci_bus_id", 0)),
          int(getattr(p, "pci_device_id", 0)), str(getattr(p, "uuid", "")))
    seen = [None] * ctx.world
    dist.all_gather_object(seen, me)
    return sum(1 for x in seen if x == me) > 1


def shutdown(ctx: DistContext) -> None:
    if ctx.enabled and dist.is_initialized():
        dist.destroy_process_group()

"""Checkpoint / resume.

Reference: tf.train.Supervisor(save_model_secs=60, logdir=./train_model/) writes
``model.ckpt-<global_step>.{meta,index,data-*}`` and auto-restores the newest on restart
(construct_distribute.py:375, 385-392; the explicit restore path is broken, :330/:399,
quirk 4); inference picks the max-step .meta (construct_inference.py:35-50) and restores
by graph-rebuild order (quirk 14).

Here a checkpoint is ONE file ``train_model/ckpt-<step>.pt`` holding only tensors, ints,
floats and strings — so it loads with ``torch.load(weights_only=True)`` — with:
named parameter tensors (``layers.<i>.weight`` ...), BN running stats, optimizer slots,
step counters, the batch-stream position and the model config JSON.  Writes are atomic
(temp file + ``os.replace``) so a crash never leaves a truncated newest checkpoint.
"""
from __future__ import annotations

import json
import math
import os
import re
from typing import Any, Dict, Optional, Tuple

import torch

CKPT_DIR = "train_model"
_PAT = re.compile(r"^ckpt-(\d+)\.pt$")
FORMAT = 1


def ckpt_dir(model_dir: str) -> str:
    return os.path.join(model_dir, CKPT_DIR)


def list_checkpoints(model_dir: str):
    d = ckpt_dir(model_dir)
    if not os.path.isdir(d):
        return []
    out = []
    for f in os.listdir(d):
        m = _PAT.match(f)
        if m:
            out.append((int(m.group(1)), os.path.join(d, f)))
    return sorted(out)


def latest(model_dir: str) -> Optional[Tuple[int, str]]:
    c = list_checkpoints(model_dir)
    return c[-1] if c else None


def save(model_dir: str, step: int, state: Dict[str, Any], keep: int = 3) -> str:
    d = ckpt_dir(model_dir)
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"ckpt-{step}.pt")
    tmp = path + ".tmp"
    payload = dict(state)
    payload["format"] = FORMAT
    payload["step"] = int(step)
    torch.save(payload, tmp)
    os.replace(tmp, path)
    for s, p in list_checkpoints(model_dir)[:-keep] if keep > 0 else []:
        try:
            os.remove(p)
        except OSError:
            pass
    return path


def load(path: str, map_location="cpu") -> Dict[str, Any]:
    obj = torch.load(path, map_location=map_location, weights_only=True)
    if not isinstance(obj, dict) or obj.get("format") != FORMAT:
        raise ValueError(f"{path}: not a cloud_server_amd checkpoint")
    return obj


def full_slots(eng) -> torch.Tensor:
    """Optimizer slots for the WHOLE flat buffer.  Under the sharded "ps" strategy each
    rank owns a slice, so this is a collective (every rank must call it)."""
    if eng.sync.strategy == "ps" and eng.ctx.enabled and eng.slots.numel():
        import torch.distributed as dist
        full = torch.empty(eng.slots.shape[0], eng.flat.numel(), device=eng.slots.device)
        for i in range(eng.slots.shape[0]):
            dist.all_gather_into_tensor(full[i], eng.slots[i].contiguous())
        return full
    return eng.slots


def engine_state(eng) -> Dict[str, Any]:
    """Everything needed to resume an engine exactly where it stopped.  Collective under
    the "ps" strategy: call on every rank, write on the chief."""
    st = eng.model.export_state()
    return {
        "model": st,
        "slots": full_slots(eng).detach().cpu(),
        # flat-buffer layout of the slots (it depends on the DP strategy: "lowrank" puts
        # the dense layers last), so a resume under another strategy can re-map them
        "layout": [[n, int(o), int(math.prod(eng.model.state.shapes[n]))]
                   for n, o in eng.model.state.offsets.items()],
        "opt_id": int(eng.opt_id),
        "dstep": int(eng.dstep.item()),
        "host_step": int(eng.host_step),
        "stream_epochs": int(eng.stream.epochs),
        "config": json.dumps(eng.cfg.raw),
    }


def restore_engine(eng, obj: Dict[str, Any]) -> None:
    eng.model.import_state(obj["model"])
    slots = obj["slots"]
    layout = obj.get("layout")
    cur = eng.model.state.offsets
    if layout and slots.dim() == 2 and any(cur.get(n) != o for n, o, _ in layout):
        remap = torch.zeros(slots.shape[0], eng.flat.numel(), dtype=slots.dtype)
        for n, o, k in layout:
            if n in cur:
                remap[:, cur[n]:cur[n] + k] = slots[:, o:o + k]
        slots = remap
    if int(obj.get("opt_id", eng.opt_id)) == eng.opt_id and slots.shape[0] == eng.slots.shape[0]:
        lo, hi = eng.sync.shard_range()
        if slots.shape[1:] == eng.slots.shape[1:]:
            eng.slots.copy_(slots.to(eng.slots.device))
        elif slots.dim() == 2 and slots.shape[1] >= hi:      # full slots -> this rank's shard
            eng.slots.copy_(slots[:, lo:hi].to(eng.slots.device))
    eng.dstep.fill_(int(obj["dstep"] if "dstep" in obj else obj["step"]))
    eng.host_step = int(obj["host_step"] if "host_step" in obj else obj["step"])
    # continue the batch sequence exactly where the unbroken run would be
    eng.stream.seek(eng.host_step)

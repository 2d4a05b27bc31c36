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
    if eng.sync.sharded and eng.slots.numel():
        import torch.distributed as dist
        full = torch.empty(eng.slots.shape[0], eng.flat.numel(), device=eng.slots.device)
        for i in range(eng.slots.shape[0]):
            dist.all_gather_into_tensor(full[i], eng.slots[i].contiguous())
        return full
    return eng.slots


def full_params(eng) -> Optional[torch.Tensor]:
    """The flat parameters every OWNER currently holds, under async_ps (a collective): there
    a rank's copy of another owner's shard is a pulled one, up to 2s clocks behind, while
    the optimizer slots saved beside it are that owner's current ones — so the saved
    parameters are gathered from the owners, as ``full_slots`` gathers the slots.  None for
    the synchronous strategies (every rank's flat is current)."""
    if getattr(eng, "aps", None) is None:
        return None
    import torch.distributed as dist
    lo, hi = eng.sync.shard_range()
    full = torch.empty_like(eng.flat)
    dist.all_gather_into_tensor(full, eng.flat[lo:hi].contiguous())
    return full


def engine_state(eng) -> Dict[str, Any]:
    """Everything needed to resume an engine exactly where it stopped.  Collective under
    the "ps" / "async_ps" strategies: call on every rank, write on the chief."""
    if hasattr(eng, "flush_params"):
        eng.flush_params()                  # a deferred dense update lands first
    st = eng.model.export_state()
    full = full_params(eng)
    if full is not None:
        for k in eng.model.state.shapes:
            st[k] = eng.model.state.view(k, full).detach().clone().cpu()
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
    if hasattr(eng, "flush_params"):
        eng.flush_params()                  # no deferred update may land on restored params
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


class AsyncCheckpointer:
    """Checkpoints that cost the training stream microseconds, not a blocking save.

    The reference's Supervisor saved every 60 s from the chief (construct_distribute.py:
    385-392).  A synchronous ``torch.save`` of the sample model (18 MB of params + slots)
    stalls the step loop for tens of ms; here a save is:

    1. a device-to-device snapshot of the flat parameters, optimizer slots, BN buffers and
       step counter, ordered on the training stream (HBM copies: a few µs);
    2. a device-to-host copy of that snapshot into pinned memory on a side stream (the
       copy engine runs it beside the next training steps);
    3. ``save()`` of the payload by a background thread once the copy's event fired.

    The "ps" strategy keeps optimizer slots sharded (a collective gather) and CPU runs
    have no streams: both fall back to the synchronous ``engine_state`` path."""

    def __init__(self, eng, model_dir: str, keep: int = 3):
        import threading
        self.eng, self.model_dir, self.keep = eng, model_dir, keep
        self._threading = threading
        self.async_ok = eng.device.type == "cuda" and not eng.sync.sharded
        self._thread = None
        self._error: Optional[BaseException] = None
        self.saved = 0
        if self.async_ok:
            dev = eng.device
            self._side = torch.cuda.Stream(dev)
            self._bufs = [n for n, _ in eng.model.named_buffers()]
            srcs = [eng.flat, eng.slots, eng.dstep] + [getattr(eng.model, n) for n in self._bufs]
            self._dev = [torch.empty_like(t) for t in srcs]
            self._host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in srcs]

    def _sources(self):
        e = self.eng
        return [e.flat, e.slots, e.dstep] + [getattr(e.model, n) for n in self._bufs]

    def save(self, chief: bool) -> None:
        eng = self.eng
        if not self.async_ok:
            state = engine_state(eng)              # collective under "ps": every rank calls
            if chief:
                save(self.model_dir, eng.host_step, state, keep=self.keep)
                self.saved += 1
            return
        if not chief:
            return                                  # replicated params: the chief saves
        self.wait()
        eng.flush_params()                          # (stream-ordered) deferred update first
        main = torch.cuda.current_stream(eng.device)
        for d, s in zip(self._dev, self._sources()):
            d.copy_(s)                              # stream-ordered device snapshot
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side):
            for h, d in zip(self._host, self._dev):
                h.copy_(d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._side)
        st = eng.model.state
        meta = {
            "layout": [[n, int(o), int(math.prod(st.shapes[n]))] for n, o in st.offsets.items()],
            "opt_id": int(eng.opt_id), "host_step": int(eng.host_step),
            "stream_epochs": int(eng.stream.epochs), "config": json.dumps(eng.cfg.raw),
        }
        step = int(eng.host_step)

        def write():
            try:
                ev.synchronize()
                flat, slots, dstep = self._host[0], self._host[1], self._host[2]
                model = {n: flat[o:o + math.prod(st.shapes[n])].view(st.shapes[n]).clone()
                         for n, o in st.offsets.items()}
                for n, h in zip(self._bufs, self._host[3:]):
                    model["buffers." + n] = h.clone()
                payload = dict(meta, model=model, slots=slots.clone(), dstep=int(dstep.item()))
                save(self.model_dir, step, payload, keep=self.keep)
                self.saved += 1
            except BaseException as exc:            # surfaced by wait()
                self._error = exc

        self._thread = self._threading.Thread(target=write, name="csa-ckpt", daemon=True)
        self._thread.start()

    def wait(self) -> None:
        """Block until the pending write (if any) is on disk; re-raise its error."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            err, self._error = self._error, None
            raise RuntimeError(f"checkpoint write failed: {err!r}") from err

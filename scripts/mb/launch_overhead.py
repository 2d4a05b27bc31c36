"""Where the fixed cost of a short timed loop goes (bench --steps 20 --warmup 5).

The 20-step bench reads ~2 us/step more than the 2000-step one; at K = 20 that is ~40 us
of fixed cost per timed region.  This splits one timed region (one 20-step graph replay
bracketed by ``torch.cuda.synchronize``) into:

* host: the Python + ``hipGraphLaunch`` time of ``run_steps`` itself;
* gpu:  start -> end events recorded around the replay (what the device spends);
* wall: the bench's timed region;
* idle_sync: one synchronize on an idle device.

MB_SPIN=1 sets hipDeviceScheduleSpin on the runtime torch loads, before any context
exists (the host spins in synchronize instead of sleeping on a completion interrupt).
Env knobs of the runtime (ROC_ACTIVE_WAIT_TIMEOUT, ...) are passed through by the caller.
Prints one JSON line.
"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if os.environ.get("MB_SPIN") == "1":
    import torch as _t  # noqa: E402  (loads the runtime; no HIP call yet)
    _hip = ctypes.CDLL(os.path.join(os.path.dirname(_t.__file__), "lib", "libamdhip64.so"))
    _rc = _hip.hipSetDeviceFlags(ctypes.c_uint(1))   # hipDeviceScheduleSpin
    assert _rc == 0, f"hipSetDeviceFlags: {_rc}"

import torch  # noqa: E402

from bench import _sample_cfg  # noqa: E402
from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.runtime.engine import TrainEngine  # noqa: E402


class _A:
    optimizer = "AdagradOptimizer"
    batch = 50


def main():
    k = int(os.environ.get("MB_K", "20"))
    reps = int(os.environ.get("MB_REPS", "30"))
    eng = TrainEngine(_sample_cfg(_A), synthetic_mnist(60000, seed=0), device="cuda:0",
                      backend="hip", use_graph=True)
    eng.step()
    lead = int(os.environ.get("MB_LEAD", "0"))      # (MB_LEAD=n: an n-step graph, then k - n)
    eng.extra_group_sizes = [k] if not lead else [k - lead] + ([lead] if lead > 1 else [])
    eng.prepare_group_graph()
    eng.run_steps(4)
    eng.sync_device()
    res = {"host": [], "gpu": [], "wall": [], "idle_sync": []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the same graph replayed back to back (no synchronize in between) for ~MB_B2B_MS ms:
    # the device time per step when the GPU never idles
    b2b_ms = float(os.environ.get("MB_B2B_MS", "0"))
    if b2b_ms > 0:
        nrep = max(1, int(b2b_ms * 1e-3 / (k * 76e-6)))
        while nrep * k + eng.stream.used >= eng.stream.chunk and nrep > 1:
            nrep //= 2
        eng.sync_device()
        e0.record()
        for _ in range(nrep):
            eng.run_steps(k)
        e1.record()
        eng.sync_device()
        out_b2b = e0.elapsed_time(e1) * 1e-3 / (nrep * k)
    for _ in range(reps):
        if eng.stream.used + k >= eng.stream.chunk:
            eng.sync_device()
        t = time.perf_counter()
        eng.sync_device()
        res["idle_sync"].append(time.perf_counter() - t)
        t0 = time.perf_counter()
        e0.record()
        if lead:
            eng.run_steps(lead)             # a short graph first: the device starts sooner
            eng.run_steps(k - lead)
        else:
            eng.run_steps(k)
        t1 = time.perf_counter()
        e1.record()
        eng.sync_device()
        t2 = time.perf_counter()
        res["host"].append(t1 - t0)
        res["wall"].append(t2 - t0)
        res["gpu"].append(e0.elapsed_time(e1) * 1e-3)
    # device time of one k-step replay after the GPU idled for ~gap us (host busy-wait
    # between a synchronize and the replay): is the short loop's premium idle-dependent?
    gaps = [float(x) for x in os.environ.get("MB_GAPS_US", "").split(",") if x]
    gap_res = {}
    for gap in gaps:
        vals = []
        for _ in range(max(3, reps // 2)):
            if eng.stream.used + k >= eng.stream.chunk:
                eng.sync_device()
            eng.sync_device()
            t = time.perf_counter()
            while (time.perf_counter() - t) * 1e6 < gap:
                pass
            e0.record()
            eng.run_steps(k)
            e1.record()
            eng.sync_device()
            vals.append(e0.elapsed_time(e1) * 1e-3 / k)
        gap_res[str(int(gap))] = round(statistics.median(vals) * 1e6, 2)
    eng.check_health()
    out = {k2: round(statistics.median(v) * 1e6, 2) for k2, v in res.items()}
    if gaps:
        out["us_per_step_after_idle_gap_us"] = gap_res
    if b2b_ms > 0:
        out["b2b_ms_per_step"] = round(out_b2b * 1e3, 5)
        out["b2b_steps"] = nrep * k
    out["wall_ms_per_step"] = round(statistics.median(res["wall"]) * 1e3 / k, 5)
    out["gpu_ms_per_step"] = round(statistics.median(res["gpu"]) * 1e3 / k, 5)
    out["env"] = {e: os.environ.get(e) for e in ("MB_SPIN", "ROC_ACTIVE_WAIT_TIMEOUT", "DEBUG_CLR_GRAPH_PACKET_CAPTURE")
                  if os.environ.get(e) is not None}
    out["k"] = k
    out["lead"] = lead
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Grouped-launch prototype: fc1's forward of K packed sample-config jobs
([50 x 3920] x [3920 x 512] each, the packed launch profile) three ways, each captured in a
HIP graph and replayed back to back:

* serial   — K launches on one stream (one job after the other);
* branches — K launches on K forked streams joined at the end (how the packed graph runs
             its jobs: one branch per job);
* grouped  — ONE launch, blockIdx.z = job x k-split over a per-job argument table
             (csa_dd_group_begin / csa_dd_group_end, dense_direct.hip dd_fwd_group_kernel).

Prints one JSON line per K with µs per "all K forwards" for each form, and checks that the
grouped launch writes exactly what the K separate launches write.

    python scripts/mb/grouped_fc1.py [--ks 1,2,4,8] [--reps 300]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config  # noqa: E402
from cloud_server_amd.ops import fused as K  # noqa: E402
from cloud_server_amd.runtime.engine import TrainEngine  # noqa: E402
from cloud_server_amd.utils.streams import dedicated_stream  # noqa: E402


class Rec:
    def __init__(self, lib):
        self.lib, self.calls = lib, []

    def __getattr__(self, name):
        fn = getattr(self.lib, name)
        if name != "csa_dd_fwd":
            return fn

        def wrapped(*args):
            self.calls.append(args)
            return fn(*args)
        return wrapped


def fc1_call(eng):
    rec = Rec(eng.program.lib)
    eng.program.lib = rec
    eng.step()
    torch.cuda.synchronize()
    eng.program.lib = rec.lib
    big = [c for c in rec.calls if c[6] == 3920]        # (X, W, bias, Y, M, N, K, ...)
    assert big, "no fc1 forward recorded"
    return big[0]


def find_tensor(eng, ptr):
    """The engine tensor whose storage starts at ``ptr`` (the recorded Y pointer)."""
    seen = []
    for u in eng.program.units:
        for v in vars(u).values():
            if isinstance(v, torch.Tensor) and v.is_cuda and v.data_ptr() == ptr:
                return v
            seen.append(v)
    raise LookupError(f"no unit tensor at {ptr:#x}")


def timed(g, reps):
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    lib = K.load()
    engines, calls = [], []
    kmax = max(int(x) for x in a.ks.split(","))
    for j in range(kmax):
        cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-4,
                                      options={"batch_size": 50}))
        cfg.seed = j
        eng = TrainEngine(cfg, synthetic_mnist(6000, seed=j), device="cuda", backend="hip", use_graph=False,
                          packed=True)
        for _ in range(2):
            eng.step()
        engines.append(eng)
        calls.append(fc1_call(eng))
    side = [dedicated_stream(torch.device("cuda", 0)) for _ in range(kmax)]
    cap = dedicated_stream(torch.device("cuda", 0))

    def launch(args, st):
        return lib.csa_dd_fwd(*args[:-1], st)

    for k in [int(x) for x in a.ks.split(",")]:
        cs = calls[:k]
        outs = [c[3] for c in cs]                       # Y pointers
        ys = [e.program.units[2].y if hasattr(e.program.units[2], "y") else None for e in engines[:k]]
        res = {"K": k}
        # correctness: grouped == separate (the split-K partials land with atomics in the same
        # order class; compare after zeroing Y)
        graphs = {}
        for form in ("serial", "branches", "grouped"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
                st = torch.cuda.current_stream()
                if form == "serial":
                    for c in cs:
                        K.check(launch(c, st.cuda_stream), "dd_fwd")
                elif form == "branches":
                    for j, c in enumerate(cs):
                        side[j].wait_stream(st)
                        with torch.cuda.stream(side[j]):
                            K.check(launch(c, side[j].cuda_stream), "dd_fwd")
                        st.wait_stream(side[j])
                else:
                    lib.csa_dd_group_begin()
                    for c in cs:
                        K.check(launch(c, st.cuda_stream), "dd_fwd(record)")
                    K.check(lib.csa_dd_group_end(st.cuda_stream), "dd_group_end")
            graphs[form] = g
        for form, g in graphs.items():
            res[f"{form}_us"] = round(timed(g, a.reps), 2)
        res["us_per_job"] = {f: round(res[f"{f}_us"] / k, 2) for f in graphs}
        print(json.dumps(res), flush=True)
        del ys, outs
    # numerics: the grouped launch writes what the separate launches write (outputs zeroed
    # first: split-K forwards accumulate with atomics)
    cs = calls[:kmax]
    ys = [find_tensor(e, c[3]) for e, c in zip(engines, cs)]
    for y in ys:
        y.zero_()
    for c in cs:
        K.check(launch(c, torch.cuda.current_stream().cuda_stream), "dd_fwd")
    torch.cuda.synchronize()
    ref = [y.clone() for y in ys]
    for y in ys:
        y.zero_()
    lib.csa_dd_group_begin()
    for c in cs:
        K.check(launch(c, torch.cuda.current_stream().cuda_stream), "dd_fwd(record)")
    K.check(lib.csa_dd_group_end(torch.cuda.current_stream().cuda_stream), "dd_group_end")
    torch.cuda.synchronize()
    worst = max(float((y - r).abs().max() / (r.abs().max() + 1e-12)) for y, r in zip(ys, ref))
    print(json.dumps({"grouped_vs_separate_max_rel_diff": worst, "jobs": kmax}), flush=True)
    if worst > 1e-5:
        raise SystemExit("grouped launch differs from the separate launches")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""Per-workgroup stamps of the one-GPU step's launches INSIDE the captured graph (the bench
program, not isolated replays): the pair forward (start / end), head_dgrad (six phase
stamps) and the carrying launch (start / end, by segment), on one device clock
(s_memrealtime, 100 MHz), relative to the pair forward's first workgroup.

    python scripts/mb/graph_life.py [--warm 300] [--edges 700,828,1808]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config  # noqa: E402
from cloud_server_amd.runtime.engine import TrainEngine  # noqa: E402


def span(t, lo, hi, t0):
    s, e = (t[lo:hi, 0] - t0) / 100.0, (t[lo:hi, -1] - t0) / 100.0
    return (f"start {float(s.min()):6.2f}..{float(s.max()):6.2f}  end {float(e.min()):6.2f}..{float(e.max()):6.2f}"
            f"  life mean {float((e - s).mean()):5.2f} max {float((e - s).max()):5.2f} us")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=int, default=300)
    ap.add_argument("--edges", default="700,828,1808")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-4,
                                  options={"batch_size": 50}))
    eng = TrainEngine(cfg, synthetic_mnist(60000, seed=0), device="cuda", backend="hip")
    for _ in range(a.warm):
        eng.step()
    torch.cuda.synchronize()
    lib = eng.program.lib
    ew = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
    dd = torch.zeros(2 * 8192, dtype=torch.int64, device="cuda")
    du = torch.zeros(16 * 1024, dtype=torch.int64, device="cuda")
    cv = torch.zeros(2 * 2048, dtype=torch.int64, device="cuda")
    cp = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
    hd = torch.zeros(8 + 8 * 2048, dtype=torch.int64, device="cuda")
    for rep in range(a.reps):
        for b in (cv, cp, hd, ew, dd, du):
            b.zero_()
        lib.csa_cpv_life_debug(cv.data_ptr()); lib.csa_cp_life_debug(cp.data_ptr()); lib.csa_head_debug(hd.data_ptr())
        lib.csa_chain_head_debug(hd.data_ptr())
        lib.csa_ew_life_debug(ew.data_ptr()); lib.csa_dd_life_debug(dd.data_ptr()); lib.csa_du_debug(du.data_ptr())
        eng.step()                                   # one replay of the captured step graph
        torch.cuda.synchronize()
        lib.csa_cpv_life_debug(None); lib.csa_cp_life_debug(None); lib.csa_head_debug(None)
        lib.csa_chain_head_debug(None)
        lib.csa_ew_life_debug(None); lib.csa_dd_life_debug(None); lib.csa_du_debug(None)
        c = cv.view(-1, 2).double().cpu(); c = c[c[:, 0] > 0]
        p = cp.view(-1, 2).double().cpu(); p = p[: int((p[:, 0] > 0).sum())]
        h = hd[8:].view(-1, 8).double().cpu(); h = h[h[:, 0] > 0][:, :6]
        t0 = float(c[:, 0].min())
        print(f"== replay {rep}: step span {(float(p[:, 1].max()) - t0) / 100:.2f} us (pair fwd first start -> carrier last end)")
        print(f"  pair fwd   {c.shape[0]:5d} wg  {span(c, 0, c.shape[0], t0)}")
        e_ = ew.view(-1, 2).double().cpu(); e_ = e_[e_[:, 0] > 0]
        print(f"  bn_act     {e_.shape[0]:5d} wg  {span(e_, 0, e_.shape[0], t0)}")
        dv = dd.view(-1, 2).double().cpu()
        d1, d2 = dv[:4096], dv[4096:]
        d1, d2 = d1[d1[:, 0] > 0], d2[d2[:, 0] > 0]
        print(f"  fc1 fwd    {d1.shape[0]:5d} wg  {span(d1, 0, d1.shape[0], t0)}")
        print(f"  fc2 fwd    {d2.shape[0]:5d} wg  {span(d2, 0, d2.shape[0], t0)}")
        print(f"  head_dgrad {h.shape[0]:5d} wg  {span(h, 0, h.shape[0], t0)}")
        ph = (h[:, 1:] - h[:, :-1]) / 100.0
        print("     phases mean (us): input landed {:.2f} | logits {:.2f} | softmax+dh {:.2f} | dX dot {:.2f} | "
              "store {:.2f}".format(*[float(ph[:, k].mean()) for k in range(5)]))
        uf = du.view(-1, 16).double().cpu()
        uf = uf[uf[:, 0] > 0]
        u_ = uf[:, [0, 6]]
        print(f"  fc1 dgrad  {u_.shape[0]:5d} wg  {span(u_, 0, u_.shape[0], t0)}")
        if uf.shape[0]:
            ph = [(uf[:, k + 1] - uf[:, k]) / 100.0 for k in range(6)]
            print("     phases mean (us): dY staged {:.2f} | W landed {:.2f} | MFMA {:.2f} | fold {:.2f} | "
                  "transform+dX {:.2f} | BN stats {:.2f}".format(*[float(x.mean()) for x in ph]))
        edges = [0] + [int(x) for x in a.edges.split(",") if x] + [p.shape[0]]
        for lo, hi in zip(edges, edges[1:]):
            if hi > lo:
                print(f"  carrier [{lo:4d},{hi:4d})  {span(p, lo, hi, t0)}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""Per-kernel micro-benchmarks of the HIP step program (GPU).

Builds the sample-config engine, then times each kernel launch of one training step in
isolation: the step's launch list is recorded once, and each launch is replayed N times
back to back (plain stream launches, event-timed).  Output: one line per launch with
µs/launch.  Run: python scripts/microbench.py [--reps 200] [--batch 50]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config  # noqa: E402
from cloud_server_amd.ops import fused as K  # noqa: E402
from cloud_server_amd.runtime.engine import TrainEngine  # noqa: E402


class Recorder:
    """Wraps the ctypes library: records (name, fn, args) of every csa_* call."""

    def __init__(self, lib):
        self.lib = lib
        self.calls = []

    def __getattr__(self, name):
        fn = getattr(self.lib, name)
        if (not name.startswith("csa_") or name.endswith(("_splits", "_slabs", "_nslab", "_ws", "_ok", "_rows", "_grid"))
                or name.startswith("csa_set_") or name in ("csa_deterministic", "csa_packed")):
            return fn

        def wrapped(*args):
            self.calls.append((name, fn, args))
            return fn(*args)
        return wrapped


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--packed", action="store_true", help="the packed (multi-tenant) launch profile")
    a = ap.parse_args()
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer",
                                  options={"batch_size": a.batch}))
    eng = TrainEngine(cfg, synthetic_mnist(6000), device="cuda", backend="hip", use_graph=False,
                      packed=a.packed)
    for _ in range(3):
        eng.step()
    rec = Recorder(eng.program.lib)
    eng.program.lib = rec
    eng.step()
    torch.cuda.synchronize()
    eng.program.lib = rec.lib
    if a.packed:
        rec.lib.csa_set_packed(1)       # replays outside the program's scope keep its shapes
    total = 0.0
    rows = []
    if os.environ.get("MB_GEMM"):
        dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
        for i, (name, fn, args) in enumerate(rec.calls):
            if name in ("csa_dense_fwd", "csa_dense_dgrad", "csa_dense_wgrad", "csa_conv_wgrad"):
                eng.program.lib.csa_gemm_debug(dbg.data_ptr())
                fn(*args)
                torch.cuda.synchronize()
                eng.program.lib.csa_gemm_debug(None)
                t = dbg.tolist()
                last = max(j for j in range(2, 6) if t[j]) if any(t[2:6]) else 1
                print(f"{i:2d} {name:18s} launch->k0 {t[2] - t[0] if t[2] else -1}  loop {t[6] - t[2] if t[2] else -1}"
                      f" (iters {[t[j + 1] - t[j] for j in range(2, last)]})  prefetch {t[8] - t[6]}"
                      f"  wk-reduce {t[9] - t[8]}  epilogue {t[7] - t[9]}  it0: commitA {t[10] - t[2]} commitB {t[11] - t[10]} mfma {t[12] - t[11]}")
                dbg.zero_()
    if os.environ.get("MB_CONV"):
        dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
        for i, (name, fn, args) in enumerate(rec.calls):
            if name == "csa_conv_fwd":
                for _ in range(3):
                    dbg.zero_()
                    eng.program.lib.csa_conv_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_conv_debug(None)
                t = dbg.tolist()
                print(f"{i:2d} {name:18s} conv stamps:", [t[j + 1] - t[j] for j in range(7)])
    if os.environ.get("MB_DU"):
        # per-block stamps (100 MHz realtime): start, loads landed, ticket drawn, finisher end
        for i, (name, fn, args) in enumerate(rec.calls):
            if name.startswith("csa_dense_bwd_update"):
                grid = 4096
                dbg = torch.zeros(grid * 16, dtype=torch.int64, device="cuda")
                for _ in range(3):
                    dbg.zero_()
                    eng.program.lib.csa_du_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_du_debug(None)
                t = dbg.view(-1, 16)
                t = t[t[:, 0] > 0].double()
                t0 = t[:, 0].min()
                names = ["stage", "W landed", "mfma+update", "fold", "epilogue", "slab atomics"]
                parts = []
                for k in range(6):
                    ok = (t[:, k + 1] > 0) & (t[:, k] > 0)
                    d = (t[ok, k + 1] - t[ok, k]) / 100
                    if len(d):
                        parts.append(f"{names[k]} {d.mean():.2f}/{d.max():.2f}")
                end = (t.max() - t0) / 100
                print(f"{i:2d} {name}: blocks {len(t)} span {end:.2f} us | start spread "
                      f"{(t[:, 0].max() - t0) / 100:.2f} | " + " | ".join(parts) + " (mean/max us)")
    if os.environ.get("MB_OPT"):
        # per-block stamps (100 MHz realtime): start, main loop done, zero lists done, end
        for i, (name, fn, args) in enumerate(rec.calls):
            if name.startswith("csa_optimizer"):
                dbg = torch.zeros(4096 * 4, dtype=torch.int64, device="cuda")
                for _ in range(3):
                    dbg.zero_()
                    eng.program.lib.csa_opt_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_opt_debug(None)
                t = dbg.view(-1, 4)
                nz = t[:, 0] > 0
                idx = torch.nonzero(nz).flatten()
                t = t[nz].double()
                t0 = t[:, 0].min()
                main = t[:, 2] > 0
                st = ~main
                def q(x):
                    return f"{x.mean():.2f}/{x.max():.2f}" if len(x) else "-"
                print(f"{i:2d} {name}: blocks {len(t)} (staging {int(st.sum())}) span {(t[:, 3].max() - t0) / 100:.2f} us | "
                      f"start spread {(t[:, 0].max() - t0) / 100:.2f} | main {q((t[main, 1] - t[main, 0]) / 100)} | "
                      f"zero {q((t[main, 2] - t[main, 1]) / 100)} | meta {q((t[main, 3] - t[main, 2]) / 100)} | "
                      f"staging {q((t[st, 3] - t[st, 0]) / 100)} (mean/max us); block0 end {(t[0, 3] - t0) / 100:.2f}")
                mt = (t[:, 1] - t[:, 0]) / 100
                top = torch.argsort(mt, descending=True)[:6]
                print("     slowest main loops (block: us):", [(int(idx[j]), round(float(mt[j]), 2)) for j in top])
    if os.environ.get("MB_CP"):
        dbg = torch.zeros(24, dtype=torch.int64, device="cuda")
        for i, (name, fn, args) in enumerate(rec.calls):
            if name.startswith("csa_conv_pair_fwd"):
                for blk in [int(x) for x in os.environ.get("MB_CP_BLOCKS", "0").split(",")]:
                    eng.program.lib.csa_cp_debug_block(blk)
                    for _ in range(3):
                        dbg.zero_()
                        eng.program.lib.csa_cp_debug(dbg.data_ptr())
                        fn(*args)
                        torch.cuda.synchronize()
                        eng.program.lib.csa_cp_debug(None)
                    t = dbg.tolist()
                    print(f"{i:2d} {name} block {blk}: stage {t[1]-t[0]} convA {t[2]-t[1]} convB+pool {t[3]-t[2]} "
                          f"stats {t[4]-t[3]} (s_memtime ticks)")
                eng.program.lib.csa_cp_debug_block(0)
            elif name.startswith("csa_conv_pair_"):
                for _ in range(3):
                    dbg.zero_()
                    eng.program.lib.csa_cp_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_cp_debug(None)
                t = dbg.tolist()
                if "fwd" in name:
                    pass
                elif t[14] == 0:      # VALU backward (cpv_bwd_kernel)
                    print(f"{i:2d} {name}: loads {t[9]-t[8]} bn+c1 {t[10]-t[9]} route {t[11]-t[10]} "
                          f"dwB+dc1 {t[12]-t[11]} dwA {t[13]-t[12]} (s_memtime ticks)")
                else:
                    print(f"{i:2d} {name}: stage+bn {t[9]-t[8]} (loads {t[16]-t[8]} tables {t[17]-t[16]} "
                          f"stores {t[18]-t[17]} bn {t[9]-t[19]}) route {t[10]-t[9]} convA {t[11]-t[10]} dwB {t[12]-t[11]} "
                          f"dc1 {t[13]-t[12]} dwA {t[14]-t[13]} atomics {t[15]-t[14]}")
    if os.environ.get("MB_DD"):
        dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
        for i, (name, fn, args) in enumerate(rec.calls):
            if name.startswith("csa_dd_"):
                for _ in range(3):
                    dbg.zero_()
                    dbg[4] = 2 ** 62
                    eng.program.lib.csa_dd_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_dd_debug(None)
                t = dbg.tolist()
                print(f"{i:2d} {name}: block0 loop {t[1]-t[0]} reduce {t[2]-t[1]} epilogue {t[3]-t[2]} "
                      f"| block0 total {t[3]-t[0]} | all blocks span {t[5]-t[4]}  first start->b0 start {t[0]-t[4]}")
    if os.environ.get("MB_HEAD"):
        dbg = torch.zeros(8, dtype=torch.int64, device="cuda")
        for i, (name, fn, args) in enumerate(rec.calls):
            if name.startswith("csa_head_part"):
                for _ in range(3):
                    dbg.zero_()
                    eng.program.lib.csa_head_debug(dbg.data_ptr())
                    fn(*args)
                    torch.cuda.synchronize()
                    eng.program.lib.csa_head_debug(None)
                t = dbg.tolist()
                print(f"{i:2d} {name}: stage {t[1]-t[0]} labels+sync {t[2]-t[1]} logits {t[3]-t[2]} "
                      f"loss {t[4]-t[3]} dW/dh {t[5]-t[4]} | total {t[5]-t[0]}")
    if os.environ.get("MB_FWD_LIFE"):
        # VALU pair forward: per-workgroup start / end (s_memrealtime, 100 MHz)
        for i, (name, fn, args) in enumerate(rec.calls):
            if name != "csa_conv_pair_fwd":
                continue
            life = torch.zeros(2 * 8192, dtype=torch.int64, device="cuda")
            for _ in range(3):
                life.zero_()
                eng.program.lib.csa_cpv_life_debug(life.data_ptr())
                fn(*args)
                torch.cuda.synchronize()
                eng.program.lib.csa_cpv_life_debug(None)
            t = life.view(-1, 2).double().cpu()
            t = t[t[:, 0] > 0]
            t0 = float(t[:, 0].min())
            st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
            print(f"{i:2d} {name}: {t.shape[0]} blocks, starts 0..{float(st.max()):.2f} us, ends "
                  f"{float(en.min()):.2f}..{float(en.max()):.2f} us | life mean {float((en - st).mean()):.2f} "
                  f"max {float((en - st).max()):.2f}")
    if os.environ.get("MB_HD"):
        # head_dgrad: per-workgroup stamps (start | logits | softmax + dh | dX), 100 MHz
        for i, (name, fn, args) in enumerate(rec.calls):
            if name != "csa_head_dgrad":
                continue
            nblk = 4096
            dbg = torch.zeros(8 + 4 * nblk, dtype=torch.int64, device="cuda")
            for _ in range(3):
                dbg.zero_()
                eng.program.lib.csa_head_debug(dbg.data_ptr())
                fn(*args)
                torch.cuda.synchronize()
                eng.program.lib.csa_head_debug(None)
            t = dbg[8:].view(nblk, 4).double().cpu()
            t = t[t[:, 0] > 0]
            t0 = float(t[:, 0].min())
            st, en = (t[:, 0] - t0) / 100.0, (t[:, 3] - t0) / 100.0
            ph = (t[:, 1:] - t[:, :-1]) / 100.0
            print(f"{i:2d} {name}: {t.shape[0]} blocks, starts 0..{float(st.max()):.2f} us, ends "
                  f"{float(en.min()):.2f}..{float(en.max()):.2f} us | life mean {float((en - st).mean()):.2f} "
                  f"max {float((en - st).max()):.2f} | phases mean loads+logits {float(ph[:, 0].mean()):.2f} "
                  f"softmax+dh {float(ph[:, 1].mean()):.2f} dX {float(ph[:, 2].mean()):.2f} us")
    # horizontal fusion: the deferred dense updates are host-side records that the pair
    # backward consumes, so every replay of that launch re-records them first
    defers = [(fn, args) for name, fn, args in rec.calls if name == "csa_dense_update_defer"]
    if os.environ.get("MB_HF_ONLY"):        # e.g. MB_HF_ONLY=0: carry only the first deferred segment
        keep = {int(x) for x in os.environ["MB_HF_ONLY"].split(",")}
        defers = [d for i, d in enumerate(defers) if i in keep]
    host_only = ("csa_dense_update_defer", "csa_dense_update_clear", "csa_dense_update_pending")

    def call(name, fn, args):
        if name == "csa_conv_pair_bwd":
            for dfn, dargs in defers:
                dfn(*dargs)
        fn(*args)

    if os.environ.get("MB_HF"):
        # horizontal fusion: the pair backward alone, the deferred updates alone (their own
        # launches), and the pair backward carrying them
        lib = eng.program.lib
        pb = [(fn, args) for name, fn, args in rec.calls if name == "csa_conv_pair_bwd"][0]
        tabs = [(fn, args) for name, fn, args in rec.calls if name == "csa_conv_pair_bn_tab"]
        # MB_TAIL=1: the pair-backward tail too (its plan is consumed by each launch)
        tails = [(fn, args) for name, fn, args in rec.calls if name == "csa_conv_pair_tail_set"]
        tails = tails if os.environ.get("MB_TAIL") == "1" else []
        if tabs or tails:                     # the BN-table pointer is consumed by each launch
            pb0 = pb

            def _pb(*args):
                for tfn, targs in tails[-1:] + tabs[-1:]:
                    tfn(*targs)
                pb0[0](*args)
            pb = (_pb, pb0[1])

        def timed(f):
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                f()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) * 1e3 / a.reps

        def pair_alone():
            lib.csa_dense_update_clear()
            pb[0](*pb[1])

        def upd_alone():
            for dfn, dargs in defers:
                dfn(*dargs)
            lib.csa_dense_update_flush(None)

        def fused():
            for dfn, dargs in defers:
                dfn(*dargs)
            pb[0](*pb[1])
        print(f"HF: pair alone {timed(pair_alone):.2f} us | updates alone {timed(upd_alone):.2f} us | "
              f"pair + updates in one launch {timed(fused):.2f} us")
        cdbg = torch.zeros(24, dtype=torch.int64, device="cuda")
        # every workgroup's start / end in the carrying launch: who is on the critical path
        life = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
        for _ in range(3):
            life.zero_()
            lib.csa_cp_life_debug(life.data_ptr())
            fused()
            torch.cuda.synchronize()
            lib.csa_cp_life_debug(None)
        lv = life.view(-1, 2).cpu()
        nblk = int((lv[:, 0] > 0).sum())
        lv = lv[:nblk].double()
        t0 = lv[:, 0].min()
        st, en = (lv[:, 0] - t0) / 100.0, (lv[:, 1] - t0) / 100.0      # us
        npair = int(os.environ.get("MB_NPAIR", "700"))
        segs = [("pair", 0, npair)]
        # deferred segments follow in record order, then the tail
        print(f"  life: {nblk} workgroups, launch span {float(en.max()):.2f} us")
        edges = [int(x) for x in os.environ.get("MB_EDGES", "").split(",") if x] or []
        bounds = [0, npair] + edges + [nblk]
        for k in range(len(bounds) - 1):
            lo, hi = bounds[k], bounds[k + 1]
            if hi <= lo:
                continue
            s_, e_ = st[lo:hi], en[lo:hi]
            print(f"    blocks [{lo},{hi}): start {float(s_.min()):.2f}..{float(s_.max()):.2f} "
                  f"end {float(e_.min()):.2f}..{float(e_.max()):.2f} life mean {float((e_ - s_).mean()):.2f} "
                  f"max {float((e_ - s_).max()):.2f} us")
        q = torch.quantile(en, torch.tensor([0.5, 0.9, 0.99], dtype=torch.float64))
        print(f"    block ends p50/p90/p99 {q[0]:.2f}/{q[1]:.2f}/{q[2]:.2f} us")
        # the carried update workgroups' own stamps (segment-local numbering: carry ONE
        # segment, MB_HF_ONLY, so that they do not collide)
        if len(defers) == 1:
            cdu = torch.zeros(4096 * 16, dtype=torch.int64, device="cuda")
            for _ in range(3):
                cdu.zero_()
                lib.csa_cp_du_debug(cdu.data_ptr())
                fused()
                torch.cuda.synchronize()
                lib.csa_cp_du_debug(None)
            t = cdu.view(-1, 16)
            t = t[t[:, 0] > 0].double()
            d = lambda k1, k0: ((t[:, k1] - t[:, k0]) / 100)
            print(f"  carried segment: blocks {len(t)} | stage {d(1, 0).mean():.2f} | W {d(2, 1).mean():.2f} | "
                  f"half 0 MFMA+update {d(7, 2).mean():.2f} | half 1 dY staged {d(4, 7).mean():.2f} | half 1 W {d(5, 4).mean():.2f} | "
                  f"half 1 MFMA+update {d(8, 5).mean():.2f} | bias {d(3, 8).mean():.2f} | store issue {d(6, 3).mean():.2f} | "
                  f"life {d(6, 0).mean():.2f} (mean us)")
        # MB_CP_BLOCKS=0,350,699: whose stamps (pair workgroups come first in both launches)
        for blk in [int(x) for x in os.environ.get("MB_CP_BLOCKS", "0").split(",")]:
            lib.csa_cp_debug_block(blk)
            for label, f in (("pair alone", pair_alone), ("pair + updates", fused)):
                for _ in range(3):
                    cdbg.zero_()
                    lib.csa_cp_debug(cdbg.data_ptr())
                    f()
                    torch.cuda.synchronize()
                    lib.csa_cp_debug(None)
                t = cdbg.tolist()
                print(f"  {label} block {blk}: loads {t[16]-t[8]} tables {t[17]-t[16]} stores {t[18]-t[17]} "
                      f"bn {t[9]-t[19]} route {t[10]-t[9]} convA {t[11]-t[10]} dwB {t[12]-t[11]} dc1 {t[13]-t[12]} "
                      f"dwA {t[14]-t[13]} atomics {t[15]-t[14]} | total {t[15]-t[8]} (s_memtime ticks)")
        lib.csa_cp_debug_block(0)
        # per-block stamps of the update-only launches (100 MHz realtime: start, dY staged,
        # W landed, MFMA + update done, stores issued)
        dbg = torch.zeros(4096 * 16, dtype=torch.int64, device="cuda")
        for dfn, dargs in defers:
            dbg.zero_()
            lib.csa_du_debug(dbg.data_ptr())
            dfn(*dargs)
            lib.csa_dense_update_flush(None)
            torch.cuda.synchronize()
            lib.csa_du_debug(None)
            t = dbg.view(-1, 16)
            t = t[t[:, 0] > 0].double()
            t0 = t[:, 0].min()
            d = lambda k1, k0: ((t[:, k1] - t[:, k0]) / 100)
            print(f"  segment K={dargs[4]} N={dargs[5]}: blocks {len(t)} span {(t[:, 6].max() - t0) / 100:.2f} us | "
                  f"start spread {(t[:, 0].max() - t0) / 100:.2f} | stage {d(1, 0).mean():.2f}/{d(1, 0).max():.2f} | "
                  f"W {d(2, 1).mean():.2f}/{d(2, 1).max():.2f} | mfma+upd {d(3, 2).mean():.2f}/{d(3, 2).max():.2f} | "
                  f"store issue {d(6, 3).mean():.2f}/{d(6, 3).max():.2f} | block life {d(6, 0).mean():.2f}/{d(6, 0).max():.2f} (mean/max us)")
            if bool((t[:, 5] > 0).all()):         # update-only bodies: the second column half
                print(f"    half 0 MFMA+update {d(4, 2).mean():.2f} | half 1 W {d(5, 4).mean():.2f} | "
                      f"half 1 MFMA+update + bias {d(3, 5).mean():.2f} (mean us)")
    for i, (name, fn, args) in enumerate(rec.calls):
        if name in host_only:
            continue
        for _ in range(5):
            call(name, fn, args)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            call(name, fn, args)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        total += us
        rows.append((i, name, us))
    for i, name, us in rows:
        print(f"{i:2d} {name:24s} {us:8.2f} us")
    print(f"sum of isolated launches: {total:.1f} us")
    # whole step, graph replay
    eng2 = TrainEngine(cfg, synthetic_mnist(6000), device="cuda", backend="hip", use_graph=True)
    for _ in range(20):
        eng2.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        eng2.step()
    e.record()
    torch.cuda.synchronize()
    print(f"graph step: {s.elapsed_time(e) * 1e3 / a.reps:.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())

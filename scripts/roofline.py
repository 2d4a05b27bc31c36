#!/usr/bin/env python3
"""Roofline table of the HIP step kernels from two rocprofv3 --pmc passes over
scripts/microbench.py plus its isolated per-launch timings.

Usage: python scripts/roofline.py <pmcA dir> <pmcB dir> <micro.txt> > profiles/r2_roofline.md
pass A: FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE
pass B: WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES
Peaks used: HBM3E 8.0 TB/s; f32 MFMA 157.3 TFLOP/s dense (256 CU x 4 SIMD x 256 flop/clk
x 2.4 GHz / 4 for 16x16x4 f32 ... quoted from MI355X_MICROARCH.md).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

HBM_TBS = 8.0
F32_MFMA_TFLOPS = 157.3


def load(d):
    """{kernel: [(grid, {counter: [values]}) in order of first appearance]} — launches that
    share a kernel symbol (the two dense layers) are told apart by their grid size."""
    out = defaultdict(dict)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            rows = list(csv.DictReader(f))
        per = {}
        for r in rows:
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"], r["Grid_Size"])
            per.setdefault(key, {})
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (_, name, grid), cs in sorted(per.items()):
            short = re.sub(r"^void |\(.*$", "", name)
            short = re.sub(r"<.*", "", short).replace("csa::", "")
            g = out[short].setdefault(grid, defaultdict(list))
            for k, v in cs.items():
                g[k].append(v)
    return {k: list(v.values()) for k, v in out.items()}


def main():
    a, b, micro = load(sys.argv[1]), load(sys.argv[2]), sys.argv[3]
    times = []
    for line in open(micro):
        m = re.match(r"\s*(\d+)\s+(csa_\w+)\s+([\d.]+) us", line)
        if m:
            times.append((int(m.group(1)), m.group(2), float(m.group(3))))
    kmap = {"csa_conv_pair_fwd": "cpv_fwd_kernel", "csa_conv_pair_bwd": "conv_pair_bwd_kernel",
            "csa_head_row": "head_row_kernel", "csa_dense_bwd_update_head": "dense_bwd_update_kernel",
            "csa_dense_bwd_grad_head": "dense_bwd_update_kernel",
            "csa_bn_act_apply": "bn_act_apply_kernel", "csa_dense_fwd": "gemm_f32_kernel",
            "csa_head_part": "head_part_kernel", "csa_head_part2": "head_part_kernel", "csa_dense_bwd": "gemm_pair_kernel",
            "csa_optimizer2": "optim_kernel", "csa_optimizer2s": "optim_kernel", "csa_dd_fwd": "dd_fwd_kernel", "csa_dd_dgrad": "dd_dgrad_kernel",
            "csa_dd_wgrad": "dd_wgrad_kernel", "csa_dense_bwd_update": "dense_bwd_update_kernel",
            "csa_dense_bwd_dgrad": "dense_bwd_update_kernel", "csa_head_dgrad": "head_dgrad_kernel"}
    # the pair backward carrying the deferred dense updates (horizontal fusion)
    if "conv_pair_bwd_upd_kernel" in a:
        kmap["csa_conv_pair_bwd"] = "conv_pair_bwd_upd_kernel"
    print("| # | launch | µs (isolated) | HBM read MB | HBM write MB | achieved TB/s | % of 8 TB/s | "
          "f32 MFMA GFLOP | TFLOP/s | % of 157 TF |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    seen = defaultdict(int)
    for i, name, us in times:
        k = kmap.get(name, name)
        la, lb = a.get(k, []), b.get(k, [])
        j = seen[k]
        ca = la[j] if j < len(la) else {}
        cb = lb[j] if j < len(lb) else {}
        # several launches share a kernel symbol (two dense layers): take the i-th distinct
        # dispatch size class by order of appearance — report the mean when ambiguous
        fetch = sum(ca.get("FETCH_SIZE", [0])) / max(len(ca.get("FETCH_SIZE", [])), 1) / 1024
        write = sum(cb.get("WRITE_SIZE", [0])) / max(len(cb.get("WRITE_SIZE", [])), 1) / 1024
        mops = sum(ca.get("SQ_INSTS_VALU_MFMA_MOPS_F32", [0])) / max(len(ca.get("SQ_INSTS_VALU_MFMA_MOPS_F32", [])), 1)
        gflop = mops * 512 / 1e9
        tbs = (fetch + write) / 1e6 / (us * 1e-6) if us else 0
        tf = gflop / 1e3 / (us * 1e-6) if us else 0
        print(f"| {i} | {name} | {us:.2f} | {fetch:.2f} | {write:.2f} | {tbs:.2f} | {100 * tbs / HBM_TBS:.0f}% | "
              f"{gflop:.3f} | {tf:.1f} | {100 * tf / F32_MFMA_TFLOPS:.1f}% |")
        seen[k] += 1
    print("\nCounters are means over each launch's dispatches (isolated back-to-back replays, so "
          "operands re-read across replays may hit L2/MALL: HBM bytes are a lower bound).")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Concurrency of a rocprofv3 kernel trace: how much of the GPU's busy time the kernels
overlap, per-kernel mean duration, and each kernel's occupancy limit on a CDNA4 CU.

Usage: python scripts/trace_overlap.py <rocpd .db | dir> [--filter csa::] > profiles/x.md

Columns: mean µs under this run's concurrency, WGs, WG size, VGPR/AGPR, LDS bytes,
WG/CU = resident workgroups per CU allowed by LDS (160 KiB), VGPRs (512 per SIMD lane,
4 SIMDs) and the 32-wave CU limit; "CU-µs" = mean µs × min(1, WGs / (256 × WG/CU)) × 256,
the share of the chip a dispatch holds for its duration (what packing can never hide).
"""
from __future__ import annotations

import argparse
import glob
import os
import sqlite3
import sys
from collections import defaultdict

CUS, LDS_CU, VGPR_LANE, WAVES_CU = 256, 160 * 1024, 512, 32


def load(path: str):
    c = sqlite3.connect(path)
    return c.execute(
        "select s.kernel_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x, "
        "s.arch_vgpr_count, s.accum_vgpr_count, s.group_segment_size "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()


def wg_per_cu(wg: int, vgpr: int, agpr: int, lds: int) -> int:
    waves = max(1, (wg + 63) // 64)
    regs = max(8, vgpr + agpr)
    per_simd = VGPR_LANE // regs
    by_vgpr = (per_simd * 4) // waves
    by_lds = LDS_CU // lds if lds else 1 << 30
    by_waves = WAVES_CU // waves
    return max(0, min(by_vgpr, by_lds, by_waves))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    paths = [a.path] if a.path.endswith(".db") else glob.glob(os.path.join(a.path, "**/*.db"), recursive=True)
    rows = []
    for p in paths:
        rows += load(p)
    rows = [r for r in rows if a.filter in r[0]]
    if not rows:
        print("no dispatches")
        return 1
    rows.sort(key=lambda r: r[1])
    busy, cur_s, cur_e, total = 0, None, None, 0
    for r in rows:
        s, e = r[1], r[2]
        total += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][2] - rows[0][1]
    agg = defaultdict(lambda: [0, 0.0, None])
    for name, s, e, grid, wg, vg, ag, lds in rows:
        v = agg[name]
        v[0] += 1
        v[1] += (e - s) / 1e3
        v[2] = (grid // max(wg, 1), wg, vg, ag, lds)
    print(f"dispatches {len(rows)}, span {span / 1e3:.1f} µs, busy (union) {busy / 1e3:.1f} µs "
          f"({100 * busy / max(span, 1):.1f}% of span), kernel time {total / 1e3:.1f} µs, "
          f"mean concurrency while busy {total / max(busy, 1):.2f}\n")
    print("| kernel | calls | mean µs | WGs | WG size | VGPR | AGPR | LDS B | WG/CU | CU-µs |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    cu_total = 0.0
    for name, (n, t, (wgs, wg, vg, ag, lds)) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        per = wg_per_cu(wg, vg, ag, lds)
        mean = t / n
        frac = min(1.0, wgs / max(CUS * per, 1))
        cu_us = mean * frac * CUS
        cu_total += cu_us * n
        short = name.split("(")[0]
        short = short if len(short) < 70 else short[:67] + "..."
        print(f"| `{short}` | {n} | {mean:.2f} | {wgs} | {wg} | {vg} | {ag} | {lds} | {per} | {cu_us:.0f} |")
    print(f"\nCU-µs total {cu_total:.0f} = {cu_total / CUS:.1f} µs of the whole chip "
          f"({100 * cu_total / CUS / max(busy / 1e3, 1e-9):.0f}% of busy time)")
    return 0


if __name__ == "__main__":
    sys.exit(main())

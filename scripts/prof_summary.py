#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace (rocpd SQLite ``.db`` or ``*kernel_stats.csv``).

Usage: python scripts/prof_summary.py <db-or-dir> [--steps N] [--top K] > profiles/x.md
Prints a markdown table: kernel, calls, total µs, mean µs, share; with ``--steps`` also
the per-step device time (sum of kernel time / N).
"""
from __future__ import annotations

import argparse
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def load_db(path: str):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select s.kernel_name, d.end - d.start, d.grid_size_x * d.grid_size_y * d.grid_size_z, "
        "d.workgroup_size_x * d.workgroup_size_y * d.workgroup_size_z, "
        "s.arch_vgpr_count, s.accum_vgpr_count, s.group_segment_size "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    paths = [a.path] if a.path.endswith(".db") else glob.glob(os.path.join(a.path, "**/*.db"), recursive=True)
    rows = []
    for p in paths:
        rows += load_db(p)
    agg = defaultdict(lambda: [0, 0.0, 0, 0, 0, 0, 0])
    for name, ns, grid, wg, vg, ag, lds in rows:
        if a.filter and a.filter not in name:
            continue
        e = agg[name]
        e[0] += 1
        e[1] += ns / 1e3
        # grid sizes are in work-items per dimension: workgroups = product(grid) / product(wg)
        e[2], e[3], e[4], e[5], e[6] = grid // max(wg, 1), wg, vg, ag, lds
    total = sum(v[1] for v in agg.values())
    print(f"| kernel | calls | total µs | mean µs | share | WGs | WG size | VGPR | AGPR | LDS B |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        short = name if len(name) < 90 else name[:87] + "..."
        print(f"| `{short}` | {v[0]} | {v[1]:.1f} | {v[1] / v[0]:.2f} | {100 * v[1] / max(total, 1e-9):.1f}% "
              f"| {v[2]} | {v[3]} | {v[4]} | {v[5]} | {v[6]} |")
    print(f"\nTotal kernel time: {total:.1f} µs over {sum(v[0] for v in agg.values())} dispatches")
    if a.steps:
        print(f"Per step (÷{a.steps}): {total / a.steps:.2f} µs device time")
    return 0


if __name__ == "__main__":
    sys.exit(main())

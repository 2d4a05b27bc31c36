#!/usr/bin/env python3
"""Step timeline from a rocprofv3 SQLite trace (``run_results.db``; the default output
format of this rocprofv3): like step_timeline.py, for the .db form.

    python scripts/trace_db_timeline.py <run_results.db> [--first cpv_fwd] [--skip 800] [--steps 3]"""
import argparse
import re
import sqlite3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first", default="cpv_fwd")
    ap.add_argument("--skip", type=int, default=800)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if a.first in r[0]]
    a.skip = min(a.skip, max(0, len(starts) - a.steps - 1))
    per = {}
    for k, s in enumerate(starts[:-1]):
        nxt = starts[k + 1]
        for r in rows[s:nxt]:
            nm = re.sub(r"\(.*", "", r[0])
            per.setdefault(nm, []).append(r[2] - r[1])
    for s in starts[a.skip:a.skip + a.steps]:
        nxt = starts[starts.index(s) + 1]
        t0 = rows[s][1]
        print(f"-- step: {(rows[nxt][1] - t0) / 1e3:.2f} us to the next step's first kernel")
        for r in rows[s:nxt]:
            nm = re.sub(r"\(.*", "", r[0])[:70]
            print(f"  + {(r[1] - t0) / 1e3:7.2f} {(r[2] - r[1]) / 1e3:7.2f} us  {nm}")
    steps = [(rows[starts[k + 1]][1] - rows[starts[k]][1]) / 1e3 for k in range(len(starts) - 1)]
    steps.sort()
    if steps:
        print(f"steps: {len(steps)}, median {steps[len(steps) // 2]:.2f} us, p10 {steps[len(steps) // 10]:.2f}, "
              f"p90 {steps[9 * len(steps) // 10]:.2f}")
    for nm, v in sorted(per.items(), key=lambda x: -sum(x[1])):
        v.sort()
        print(f"  median {v[len(v) // 2] / 1e3:7.2f} us  x{len(v):5d}  {nm[:70]}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

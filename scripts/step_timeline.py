#!/usr/bin/env python3
"""Timeline of a few consecutive steps from a rocprofv3 kernel trace (csv): every kernel's
start offset from the step's first kernel, duration and queue — to see what overlaps what
in a multi-stream (DP) step.

    python scripts/step_timeline.py <run_kernel_trace.csv> [--first NAME] [--skip N] [--steps K]

A step starts at each dispatch of ``--first`` (default: the pair forward)."""
import argparse
import csv


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="cpv_fwd_kernel")
    ap.add_argument("--skip", type=int, default=200)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    if len(starts) < a.skip + a.steps + 1:
        a.skip = max(0, len(starts) - a.steps - 1)
    for s in range(a.skip, a.skip + a.steps):
        i0, i1 = starts[s], starts[s + 1]
        t0 = int(rows[i0]["Start_Timestamp"])
        t1 = int(rows[i1]["Start_Timestamp"])
        print(f"-- step {s}: {(t1 - t0) / 1e3:.2f} us to the next step's first kernel")
        for r in rows[i0:i1]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            nm = r["Kernel_Name"].replace("void ", "")
            nm = nm[:nm.find("(")] if "(" in nm else nm
            print(f"  q{r['Queue_Id']:>2} +{(st - t0) / 1e3:7.2f} {(en - st) / 1e3:7.2f} us  {nm[:80]}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

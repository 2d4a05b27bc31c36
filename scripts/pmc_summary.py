#!/usr/bin/env python3
"""Per-kernel PMC summary from a rocprofv3 ``--pmc -f csv`` directory (mean per dispatch).

Columns: duration (kernel trace), waves, wave-cycles, share of wave-cycles parked on
s_waitcnt/barrier (WAIT_ANY), issue-stalled (WAIT_INST_ANY), issuing (ACTIVE_INST_ANY),
and VALU / VMEM-read / SALU instructions per wave."""
import collections
import csv
import glob
import os
import sys


def main(d):
    cc = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    rows = list(csv.DictReader(open(cc)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    seen = set()
    for r in rows:
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (r["Dispatch_Id"], k)
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("| kernel | calls | mean µs | waves | wave-cyc | wait% | stall% | active% | VALU/wave | VMEM/wave | SALU/wave |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for k, d2 in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]])):
        if not k.startswith(("csa", "void csa")):
            continue
        m = {c: sum(v) / len(v) for c, v in d2.items()}
        w = max(m.get("SQ_WAVES", 1), 1)
        wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
        name = k.replace("void ", "").split("(")[0][:70]
        print(f"| `{name}` | {len(dur[k])} | {sum(dur[k]) / len(dur[k]):.1f} | {w:.0f} | {wc:.0f} | "
              f"{100 * m.get('SQ_WAIT_ANY', 0) / wc:.0f} | {100 * m.get('SQ_WAIT_INST_ANY', 0) / wc:.0f} | "
              f"{100 * m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0f} | {m.get('SQ_INSTS_VALU', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | {m.get('SQ_INSTS_SALU', 0) / w:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1])

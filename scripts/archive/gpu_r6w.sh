#!/bin/bash
# round 6: LDS bank conflicts of the carrying launch's parts (MB_HF: pair alone / updates
# alone / both), grouped by kernel and grid size
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/lds2
cd /tmp
MB_HF=1 MB_HF_ONLY=1 timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -f csv -d "$R/gpurun_out/lds2" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/lds2.log" 2>&1 || { echo "pass failed"; tail -5 $R/gpurun_out/lds2.log; exit 7; }
cd $R && python3 - <<'PY'
import csv, glob, collections
rows = []
for p in glob.glob("gpurun_out/lds2/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
print(sorted(rows[0].keys()))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    key = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "?")))
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    bc, act = m.get("SQ_LDS_BANK_CONFLICT", 0), m.get("SQ_LDS_IDX_ACTIVE", 0)
    if act == 0: continue
    print(f"{k[0]:70s} grid {k[1]:>8s} conflict {bc:10.0f} active {act:10.0f} ratio {bc / act:.3f} lds {m.get('SQ_INSTS_LDS', 0):9.0f} waves {m.get('SQ_WAVES', 0):7.0f}")
PY

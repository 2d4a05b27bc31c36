#!/bin/bash
# round 6: LDS bank conflicts per step kernel (one PMC pass over the microbenchmark)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/lds
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -f csv -d "$R/gpurun_out/lds" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/lds.log" 2>&1 || { echo "pass failed"; tail -5 $R/gpurun_out/lds.log; exit 7; }
cd $R && python3 - <<'PY'
import csv, glob, collections
rows = []
for p in glob.glob("gpurun_out/lds/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:80]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    bc, act = m.get("SQ_LDS_BANK_CONFLICT", 0), m.get("SQ_LDS_IDX_ACTIVE", 0)
    print(f"{k:80s} conflict {bc:12.0f} idx_active {act:12.0f} ratio {bc / act if act else 0:.3f} lds_insts {m.get('SQ_INSTS_LDS', 0):10.0f}")
PY

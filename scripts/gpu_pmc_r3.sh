#!/bin/bash
# PMC pass over the isolated step launches (microbench): LDS traffic / bank conflicts and wait states.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -f csv -d "$R/gpurun_out/pmc_r3a" -o run -- python3 "$R/scripts/microbench.py" --reps 20 > "$R/gpurun_out/pmc_r3a.log" 2>&1
echo "pmc rc=$?"
cd $R && python3 - <<'PY'
import csv, glob, collections
cc = glob.glob("gpurun_out/pmc_r3a/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(cc)):
    agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "csa" not in k: continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    print(f"{k[:60]:60s} waves {w:7.0f} wavecyc/wave {m.get('SQ_WAVE_CYCLES',0)/w:8.0f} wait% {100*m.get('SQ_WAIT_ANY',0)/max(m.get('SQ_WAVE_CYCLES',1),1):5.1f} "
          f"waitLDS% {100*m.get('SQ_WAIT_INST_LDS',0)/max(m.get('SQ_WAVE_CYCLES',1),1):5.1f} LDSinst/wave {m.get('SQ_INSTS_LDS',0)/w:7.1f} "
          f"bankconf/LDSinst {m.get('SQ_LDS_BANK_CONFLICT',0)/max(m.get('SQ_INSTS_LDS',1),1):6.2f}")
PY

#!/bin/bash
# Kernel traces of the captured step (bench, 300 steps) for two env settings.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for v in 0 1; do
  rm -rf $R/gpurun_out/tr$v
  cd /tmp
  CSA_OPT_TAIL=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr$v -o run -- python3 $R/bench.py --steps 300 --warmup 50 > $R/gpurun_out/tr$v.log 2>&1 || { tail -5 $R/gpurun_out/tr$v.log; exit 3; }
  cd $R
  echo "== CSA_OPT_TAIL=$v"; tail -1 gpurun_out/tr$v.log
  f=$(find gpurun_out/tr$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:14]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2), 'us avg')
"
done

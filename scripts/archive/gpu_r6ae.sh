#!/bin/bash
# round 6: one 20-step graph vs a short lead graph + the rest (device start latency)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for lead in 0 1 2 4; do
    MB_LEAD=$lead MB_K=20 MB_REPS=30 timeout -k 10 200 python scripts/mb/launch_overhead.py > gpurun_out/lead_${lead}_$r.json 2>>gpurun_out/lead.err || exit $?
  done
done
for f in gpurun_out/lead_*.json; do echo "$f $(python3 -c "import json,sys;d=json.load(open('$f'));print(d['wall_ms_per_step'], d['gpu_ms_per_step'], d['host'])")"; done

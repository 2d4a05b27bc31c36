#!/bin/bash
# round 6: per-step device time by graph length and continuity (short timed loop vs long)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for k in 20 32 64; do
  MB_K=$k MB_B2B_MS=35 MB_REPS=20 $T 150 python scripts/mb/launch_overhead.py > gpurun_out/lo2_k$k.json 2>>gpurun_out/lo2.err || exit $?
done
CSA_WARM_MS=0 MB_K=20 MB_B2B_MS=35 MB_REPS=20 $T 150 python scripts/mb/launch_overhead.py > gpurun_out/lo2_nowarm.json 2>>gpurun_out/lo2.err || exit $?
cat gpurun_out/lo2_*.json

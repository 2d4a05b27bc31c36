#!/bin/bash
# round 6: per-step device time of a 20-step replay after an idle gap of 0 .. 20 ms
set -o pipefail
mkdir -p gpurun_out
MB_K=20 MB_REPS=20 MB_B2B_MS=35 MB_GAPS_US=0,20,100,500,2000,20000 timeout -k 10 300 python scripts/mb/launch_overhead.py > gpurun_out/lo_gap.json 2>gpurun_out/lo_gap.err || { tail -20 gpurun_out/lo_gap.err; exit 3; }
cat gpurun_out/lo_gap.json

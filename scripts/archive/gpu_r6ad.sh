#!/bin/bash
# round 6: bench 20-step timed loop — 5 vs 30 warm-up steps right before it (clock ramp?)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for w in 5 30; do
    timeout -k 10 120 python bench.py --steps 20 --warmup $w > gpurun_out/bw_${w}_$r.json 2>>gpurun_out/bw.err || exit $?
  done
done
for w in 5 30; do echo -n "warmup $w: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/bw_${w}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done

#!/bin/bash
# round 6: non-temporal activation stores (CSA_NT_OUT) — numerics with the knob on, in-graph
# stamps and alternating benches off / on
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
CSA_NT_OUT=1 $T 600 $PYT tests/test_hip_step.py tests/test_gpu_chain.py > gpurun_out/t_step.log 2>&1 || exit $?
for v in 0 1; do
  CSA_NT_OUT=$v $T 180 python scripts/mb/graph_life.py --reps 2 > gpurun_out/glife_nt$v.txt 2>&1 || exit $?
done
for r in 1 2 3; do
  for v in 0 1; do
    CSA_NT_OUT=$v $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_nt${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    CSA_NT_OUT=$v $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_nt${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done

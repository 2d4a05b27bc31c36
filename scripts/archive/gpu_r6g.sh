#!/bin/bash
# round 6: fused forward chain (fc1 fwd | fc2 fwd | head_dgrad in one launch) — numerics,
# in-graph stamps, same-box A/B against ab/r6head; production DP test at world 2
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py tests/test_gpu_dp_overlap.py > gpurun_out/t_step.log 2>&1 || exit $?
$T 180 python scripts/mb/graph_life.py > gpurun_out/glife.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export CSA_KERNEL_LIB=ab/r6head/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
unset CSA_KERNEL_LIB
$T 600 $PYT tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?

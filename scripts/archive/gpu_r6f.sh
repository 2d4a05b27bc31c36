#!/bin/bash
# round 6: pair-backward GEMM tiles interleaved two per wave — numerics, in-graph stamps,
# same-box A/B against ab/r6head (the head_dgrad commit); production DP test (restructured)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py > gpurun_out/t_step.log 2>&1 || exit $?
$T 180 python scripts/mb/graph_life.py > gpurun_out/glife.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export CSA_KERNEL_LIB=ab/r6head/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
unset CSA_KERNEL_LIB
$T 1100 $PYT --timeout 1000 tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?

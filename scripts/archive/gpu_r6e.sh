#!/bin/bash
# round 6: head_dgrad transposed logits reduction — numerics, in-graph stamps, same-box A/B
# against the round's base kernels; grouped fc1 forward prototype; production DP test
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py > gpurun_out/t_step.log 2>&1 || exit $?
$T 180 python scripts/mb/graph_life.py > gpurun_out/glife.txt 2>&1 || exit $?
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export CSA_KERNEL_LIB=ab/r6base/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
unset CSA_KERNEL_LIB
$T 300 python scripts/mb/grouped_fc1.py > gpurun_out/grouped.txt 2>&1 || exit $?
$T 1000 $PYT --timeout 900 tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?

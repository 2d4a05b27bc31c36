#!/bin/bash
# round 6: fc1 dgrad dY by LDS-DMA + one BN-channel division; the carried update's flag
# cleared by bn_act_apply (no same-address ticket) — numerics, 1-GPU A/B vs ab/r6head,
# world-1 DP programs vs the round-5 kernels (ab/r5)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py tests/test_gpu_dp_overlap.py > gpurun_out/t_step.log 2>&1 || exit $?
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then export CSA_KERNEL_LIB=ab/r6head/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
for s in allreduce:hf allreduce ps:hf; do
  for v in r5 new; do
    if [ $v = r5 ]; then export CSA_KERNEL_LIB=ab/r5/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 200 python scripts/bench_dp1.py --strategy $s > gpurun_out/dp_${v}_$s.json 2>>gpurun_out/dp.err || exit $?
  done
done
unset CSA_KERNEL_LIB
$T 180 python scripts/mb/graph_life.py --reps 1 > gpurun_out/glife.txt 2>&1 || exit $?

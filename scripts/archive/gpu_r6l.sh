#!/bin/bash
# round 6: small conv A on VALU in the pair backward (c1 recompute, dwA + bias sums in one
# pass) — numerics, pair-workgroup phases (MB_HF stamps) and the 1-GPU A/B vs ab/r6c (HEAD);
# async_ps world-1 fences skipped
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py tests/test_gpu_dp_overlap.py > gpurun_out/t_step.log 2>&1 || exit $?
for v in r6c new; do
  if [ $v = r6c ]; then export CSA_KERNEL_LIB=ab/r6c/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
  MB_HF=1 MB_CP_BLOCKS=0,350,699 $T 180 python scripts/microbench.py > gpurun_out/mbhf_$v.txt 2>&1 || exit $?
done
for r in 1 2 3; do
  for v in r6c new; do
    if [ $v = r6c ]; then export CSA_KERNEL_LIB=ab/r6c/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
unset CSA_KERNEL_LIB
for r in 1 2; do
  $T 200 python scripts/bench_dp1.py --strategy async_ps > gpurun_out/dp_apshf_$r.json 2>>gpurun_out/dp.err || exit $?
done
$T 180 python scripts/mb/graph_life.py --reps 1 > gpurun_out/glife.txt 2>&1 || exit $?

#!/bin/bash
# round 6: tail poll sleep 8 -> 1 — numerics, in-graph carrier end, 1-GPU A/B vs ab/r6e (HEAD)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_gpu_health.py tests/test_gpu_dp_overlap.py > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 3; }
tail -1 gpurun_out/t_ab.log
for v in r6e new; do
  if [ $v = r6e ]; then export CSA_KERNEL_LIB=ab/r6e/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
  $T 180 python scripts/mb/graph_life.py --reps 2 > gpurun_out/glife_ab_$v.txt 2>&1 || exit $?
  echo "$v: $(grep -E 'span' gpurun_out/glife_ab_$v.txt | tr '\n' ' ')"
  grep -E "carrier \[1808" gpurun_out/glife_ab_$v.txt
done
for r in 1 2 3; do
  for v in r6e new; do
    if [ $v = r6e ]; then export CSA_KERNEL_LIB=ab/r6e/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
for v in r6e new; do for n in 2000 20; do echo -n "$v $n: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_${n}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done; done

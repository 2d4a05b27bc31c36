#!/bin/bash
# round 6: no closing RMW in the carrier's tail (tickets zeroed by the next pair forward) —
# numerics (step, health/forced timeout, DP :hf fold, packed), in-graph tail end, A/B vs ab/r6f
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py tests/test_gpu_dp_overlap.py tests/test_gpu_platform.py -k "not production_job_loop" > gpurun_out/t_ag.log 2>&1 || { tail -30 gpurun_out/t_ag.log; exit 3; }
tail -n1 gpurun_out/t_ag.log
for v in r6f new; do
  if [ $v = r6f ]; then export CSA_KERNEL_LIB=ab/r6f/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
  $T 180 python scripts/mb/graph_life.py --reps 2 > gpurun_out/glife_ag_$v.txt 2>&1 || exit $?
  echo "$v: $(grep -E 'span' gpurun_out/glife_ag_$v.txt | tr '\n' ' ')"
  grep -E "carrier \[(0|1808)," gpurun_out/glife_ag_$v.txt
done
for r in 1 2 3; do
  for v in r6f new; do
    if [ $v = r6f ]; then export CSA_KERNEL_LIB=ab/r6f/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
for v in r6f new; do for n in 2000 20; do echo -n "$v $n: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_${n}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done; done

#!/bin/bash
# round 6: conv weight-gradient stripes 16 vs 8 vs 12 (pair atomics contention vs tail loads)
set -o pipefail
mkdir -p gpurun_out
CSA_WGRAD_STRIPES=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_step.py > gpurun_out/t_ws.log 2>&1 || { tail -20 gpurun_out/t_ws.log; exit 3; }
tail -n1 gpurun_out/t_ws.log
for r in 1 2 3; do
  for S in 16 8 12; do
    CSA_WGRAD_STRIPES=$S timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ws_${S}_2000_$r.json 2>>gpurun_out/ws.err || exit $?
    CSA_WGRAD_STRIPES=$S timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ws_${S}_20_$r.json 2>>gpurun_out/ws.err || exit $?
  done
done
for S in 16 8 12; do for n in 2000 20; do echo -n "$S $n: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/ws_${S}_${n}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done; done

#!/bin/bash
# round 6: packed K = 4 / 8 — fc1's dense blocks wide (1024 threads) vs the packed 128-column blocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_platform.py -k "packed" > gpurun_out/t_pkw.log 2>&1 || { tail -30 gpurun_out/t_pkw.log; exit 3; }
CSA_DU_WIDE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_platform.py -k "packed_hip_jobs_match_solo" > gpurun_out/t_pkw1.log 2>&1 || { tail -30 gpurun_out/t_pkw1.log; exit 3; }
for r in 1 2; do
  for k in 4 8; do
    timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pkw_n_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
    CSA_DU_WIDE=1 timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pkw_w_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
  done
done
tail -1 gpurun_out/t_pkw.log gpurun_out/t_pkw1.log
for f in gpurun_out/pkw_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done

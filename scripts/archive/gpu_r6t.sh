#!/bin/bash
# round 6: packed K = 4 / 8 — pooled rows per conv-pair workgroup in the packed profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_platform.py -k "packed_hip_jobs_match_solo" > gpurun_out/t_pk.log 2>&1 || { tail -30 gpurun_out/t_pk.log; exit 3; }
for pr in 3 4; do
  CSA_PACKED_PR=$pr timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_platform.py -k "packed_hip_jobs_match_solo" > gpurun_out/t_pk$pr.log 2>&1 || { tail -30 gpurun_out/t_pk$pr.log; exit 3; }
done
for r in 1 2; do
  for pr in 2 3 4; do
    for k in 4 8; do
      CSA_PACKED_PR=$pr timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pkr_${pr}_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
    done
  done
done
tail -1 gpurun_out/t_pk*.log
for f in gpurun_out/pkr_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done

#!/bin/bash
# round 6: packed profile with horizontal fusion by default — packed device tests, curve
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_platform.py -k "packed" > gpurun_out/t_packed.log 2>&1 || { tail -30 gpurun_out/t_packed.log; exit 3; }
tail -3 gpurun_out/t_packed.log
for k in 1 2 4 8; do
  timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pack_$k.json 2>>gpurun_out/pack.err || exit $?
done
timeout -k 10 300 python bench.py --jobs 8 --steps 1024 --warmup 128 --pack procs > gpurun_out/pack_8procs.json 2>>gpurun_out/pack.err || exit $?
for f in gpurun_out/pack_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done

#!/bin/bash
# quick sanity on the final tree: step numerics, packed, health, smoke, the driver's bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_hip_step.py tests/test_gpu_health.py tests/test_gpu_platform.py -k "not production_job_loop" > gpurun_out/sanity.log 2>&1 || { tail -20 gpurun_out/sanity.log; exit 3; }
tail -n1 gpurun_out/sanity.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 4
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/sanity_b20.json || exit 5
grep -o '"ms_per_step": [0-9.]*' gpurun_out/sanity_b20.json

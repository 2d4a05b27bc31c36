#!/bin/bash
# round 6, first GPU call: watchdog-thread probe, baseline bench, the new health and
# production-DP tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/mb/watchdog_probe.py > gpurun_out/wd_probe.jsonl 2>gpurun_out/wd_probe.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench0.json 2>gpurun_out/bench0.err || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_health.py > gpurun_out/t_health.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?

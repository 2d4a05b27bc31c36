#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_bench_contract.py -m gpu > gpurun_out/t_rehearse.log 2>&1; rc=$?
tail -5 gpurun_out/t_rehearse.log; exit $rc

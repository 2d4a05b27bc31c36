#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_image_ops.py -x -q -m gpu > gpurun_out/imgops_tests.log 2>&1
rc=$?
tail -30 gpurun_out/imgops_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_preprocess.py > gpurun_out/bench_preprocess.jsonl 2>&1 || { tail -20 gpurun_out/bench_preprocess.jsonl; exit 3; }
cat gpurun_out/bench_preprocess.jsonl
exit $rc

#!/bin/bash
# xGMI multi-process tests in suite order, twice (flag write-back fix).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4p_$i.log 2>&1
rc=$?; echo "run $i rc=$rc $(grep -E 'passed|failed' gpurun_out/r4p_$i.log | tail -1)"
[ $rc -ne 0 ] && { grep -E "AssertionError|RuntimeError" gpurun_out/r4p_$i.log | head -4 | cut -c1-600; exit $rc; }
done
exit 0

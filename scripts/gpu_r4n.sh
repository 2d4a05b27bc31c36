#!/bin/bash
# ps on RCCL inside graph capture: watchdog event query abort — with / without the NCCL event cache.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 0 1; do
TORCH_NCCL_CUDA_EVENT_CACHE=$c timeout -k 10 200 python3 -u -m pytest "tests/test_gpu_dp_overlap.py::test_ps_and_rccl_programs_match_single_gpu" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4n_$c.log 2>&1
rc=$?; echo "event_cache=$c rc=$rc $(grep -E 'passed|failed' gpurun_out/r4n_$c.log | tail -1)"
[ $rc -eq 134 ] && { grep -m2 "hipError\|HIP error" gpurun_out/r4n_$c.log; exit 134; }
[ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 134 ] && exit $rc
done
exit 0

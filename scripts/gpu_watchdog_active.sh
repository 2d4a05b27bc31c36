#!/bin/bash
# The capture-right-after-eager-collectives test with the RCCL watchdog thread ACTIVE
# (TORCH_NCCL_BLOCKING_WAIT=0: the capture group's retirement wait is exercised).
# Not part of the closing check: in that mode the round-5 watchdog abort is still possible
# (profiles/r6_notes.md) — which is why blocking-wait mode is the default.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TORCH_CPP_LOG_LEVEL=INFO TORCH_NCCL_BLOCKING_WAIT=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dp_overlap.py -x -v -s -p no:cacheprovider -k capture_right_after --timeout 200 --timeout-method thread > gpurun_out/watchdog_active.log 2>&1
rc=$?; grep -iE "passed|failed|Aborted|watchdog|Captured|exception|terminate|error" gpurun_out/watchdog_active.log | head -40; exit $rc

#!/bin/bash
# Packed-jobs segfault: the test alone, then with the pair tables off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python3 -u -X faulthandler -m pytest "tests/test_gpu_platform.py::test_packed_hip_jobs_match_solo" -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4r_a.log 2>&1
rc=$?; echo "tables on: rc=$rc $(grep -E 'passed|failed' gpurun_out/r4r_a.log | tail -1)"
[ $rc -ne 0 ] && { grep -v "^  " gpurun_out/r4r_a.log | tail -25 | cut -c1-300; exit $rc; }
exit 0

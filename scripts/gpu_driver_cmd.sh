#!/bin/bash
# The round-end driver's exact GPU-suite command, with its output kept under gpurun_out/.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/driver_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "csa-test|passed|failed|Fatal|Error" gpurun_out/driver_pytest.log | tail -15
exit $rc

#!/bin/bash
# Full GPU check: every @gpu test, smoke(), default bench.  Each GPU step time-limited;
# stop at the first crash/timeout (exit codes >1 from pytest, any from the rest).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 4; }
cat gpurun_out/bench_default.json
exit $rc

#!/bin/bash
# round 6: async_ps own push applied from the gradient / kept in a local selfbox, no
# publication at world 1 — device tests (world 1 numerics, world 2/4/8 convergence), the
# world-1 bench, and a kernel trace of it
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_gpu_dp_overlap.py -k async tests/test_gpu_xgmi.py -k "async" > gpurun_out/t_aps.log 2>&1 || exit $?
for r in 1 2; do
  $T 200 python scripts/bench_dp1.py --strategy async_ps > gpurun_out/dp_apshf_$r.json 2>>gpurun_out/dp.err || exit $?
  $T 200 python scripts/bench_dp1.py --strategy async_ps:flat > gpurun_out/dp_aps_$r.json 2>>gpurun_out/dp.err || exit $?
done
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
cd /tmp && $T 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_aps -o run -- python3 $R/scripts/bench_dp1.py --strategy async_ps --steps 1000 --warmup 100 > $R/gpurun_out/trace_aps.log 2>&1 || exit $?
cd $R && python3 scripts/prof_summary.py gpurun_out/trace_aps --steps 1100 --top 30 > gpurun_out/trace_aps.md
cat gpurun_out/dp_*.json

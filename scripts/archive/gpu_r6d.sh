#!/bin/bash
# round 6: in-graph workgroup stamps of the step; the pair forward's block phases; then the
# thread-fact / DP-overlap tests and the production DP test
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 180 python scripts/mb/graph_life.py > gpurun_out/glife.txt 2>&1 || exit $?
MB_CP=1 MB_CP_BLOCKS=0,350,699 $T 120 python scripts/microbench.py --reps 50 > gpurun_out/mb_cp.txt 2>&1 || exit $?
$T 300 $PYT tests/test_gpu_rccl_threads.py tests/test_gpu_dp_overlap.py > gpurun_out/t_thr.log 2>&1 || exit $?
$T 900 $PYT tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?
$T 300 python scripts/mb/grouped_fc1.py > gpurun_out/grouped.txt 2>&1 || exit $?

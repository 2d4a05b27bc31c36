#!/bin/bash
# round 6: where the carrier's time goes after the residency change (life stamps, new vs
# base lib), head_dgrad / pair-forward workgroup stamps, a kernel trace of the bench step;
# then the thread-fact test, DP overlap (carry ticket) and the production DP test
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
R=$GRAFT_REPO_ROOT
export MB_EDGES=828,1808
MB_HF=1 $T 120 python scripts/microbench.py --reps 200 > gpurun_out/mb_new.txt 2>&1 || exit $?
CSA_KERNEL_LIB=ab/r6base/libcsa_kernels.so MB_HF=1 $T 120 python scripts/microbench.py --reps 200 > gpurun_out/mb_base.txt 2>&1 || exit $?
MB_HD=1 MB_FWD_LIFE=1 MB_DD=1 $T 120 python scripts/microbench.py --reps 200 > gpurun_out/mb_stamps.txt 2>&1 || exit $?
export TMPDIR=/tmp
( cd /tmp && $T 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 ) || exit $?
$T 300 $PYT tests/test_gpu_rccl_threads.py tests/test_gpu_dp_overlap.py > gpurun_out/t_thr.log 2>&1 || exit $?
$T 900 $PYT tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?

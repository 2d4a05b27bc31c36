#!/bin/bash
# Round 5: the intermittent default-group watchdog abort (hipErrorCapturedEvent) came back
# once in bench_dp1 --strategy allreduce.  Does TORCH_NCCL_BLOCKING_WAIT=1 (no watchdog
# thread at all) keep capture and the DP programs working?  DP GPU tests + 3 x 4 DP benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export TORCH_NCCL_BLOCKING_WAIT=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_sync_bn.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5bw_t.txt 2>&1 || { tail -30 gpurun_out/r5bw_t.txt; exit 3; }
tail -1 gpurun_out/r5bw_t.txt
for r in 1 2 3; do
  for s in allreduce allreduce:hf ps ps:hf; do
    t0=$(date +%s.%N)
    timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $s > gpurun_out/r5bw_$s.json 2>> gpurun_out/r5bw.err || { tail -20 gpurun_out/r5bw.err; exit 6; }
    echo "run $r $s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5bw_$s.json) wall $(echo "$(date +%s.%N) - $t0" | bc)"
  done
done

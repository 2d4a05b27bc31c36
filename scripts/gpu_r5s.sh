#!/bin/bash
# Round 5: which part of the overlapped step exposes the shared-GPU stall at world 2?
# (a) no side stream (CSA_DP_OVERLAP=0); (b) the test's deterministic mode; (c) both.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp CSA_XGMI_TIMEOUT_S=3
out=gpurun_out/r5s.jsonl; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 10 200 python3 scripts/xgmi_stress.py --world 2 --steps 300 >> $out 2>> gpurun_out/r5s.err
  rc=$?; echo "$* rc=$rc"; [ $rc -gt 1 ] && { tail -5 gpurun_out/r5s.err; exit $rc; }; return 0; }
run CSA_DP_OVERLAP=0 && run CSA_DP_OVERLAP=0 && run CSA_DETERMINISTIC=1 && run CSA_DETERMINISTIC=1 && run CSA_DP_OVERLAP=0 CSA_DETERMINISTIC=1
# packed K = 8: per-kernel time under the multi-job graph
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pk -o run -- \
  python3 bench.py --jobs 8 --steps 800 --warmup 200 > gpurun_out/r5pk.log 2>&1
echo "packed prof rc=$?"

#!/bin/bash
# Round 5: the shared-GPU launch profile (no 16-wave workgroups when ranks share a GPU).
# Stress at world 2 / 3 (allreduce, ps) with it, one world-2 run without it (the stall).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export CSA_XGMI_TIMEOUT_S=3; out=gpurun_out/r5u.jsonl; : > $out
run() { local prof=$1; shift; echo "== profile=$prof $*" >> $out
  CSA_SHARED_GPU_PROFILE=$prof timeout -k 10 200 python3 scripts/xgmi_stress.py --steps 300 "$@" >> $out 2>> gpurun_out/r5u.err
  rc=$?; echo "profile=$prof $* rc=$rc"; [ $rc -gt 1 ] && exit $rc; return 0; }
run 1 --world 2 && run 1 --world 2 && run 1 --world 2 && run 1 --world 2 --strategy ps && \
run 1 --world 3 && run 1 --world 2 --strategy async_ps && run 0 --world 2

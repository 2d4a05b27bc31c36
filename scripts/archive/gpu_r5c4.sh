#!/bin/bash
# Round 5: where is the main thread when the default group's watchdog aborts? (Python
# stacks of every thread at SIGABRT: PYTHONFAULTHANDLER), overlapped all-reduce, world 1.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
for r in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 200 python3 scripts/bench_dp1.py --strategy allreduce > gpurun_out/r5c4_$r.json 2> gpurun_out/r5c4_$r.err
  rc=$?; echo "run $r rc=$rc"
  if [ $rc -eq 134 ]; then grep -v "hostname of the client\|amdgpu.ids\|frame #" gpurun_out/r5c4_$r.err | grep -A 40 "Thread 0x\|Current thread" | head -80; exit 0; fi
  [ $rc -ne 0 ] && exit $rc
done
exit 0

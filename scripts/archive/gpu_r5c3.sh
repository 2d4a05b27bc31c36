#!/bin/bash
# Round 5: DP world-1 bench runs back to back (the intermittent watchdog abort: default-group
# works retired before every capture), with the carried dense update; wall time per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
n=0; bad=0
for r in 1 2 3 4 5 6; do for s in allreduce allreduce:hf; do
  t0=$(date +%s.%N)
  timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $s > gpurun_out/r5c3_${r}_$s.json 2> gpurun_out/r5c3_${r}_$s.err
  rc=$?; t1=$(date +%s.%N); n=$((n+1)); [ $rc -ne 0 ] && bad=$((bad+1))
  echo "run $r $s rc=$rc wall=$(echo "$t1 - $t0" | bc) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5c3_${r}_$s.json)"
  [ $rc -ne 0 ] && [ $rc -ne 134 ] && exit $rc
done; done
echo "runs=$n aborted=$bad"
exit 0

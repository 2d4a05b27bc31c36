#!/bin/bash
# Round 5: tail parameter values prefetched before the wait.  Numerics, graph trace of the
# step (per-kernel means), same-box A/B against ab_old (4c08035).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5tp_t.txt 2>&1 || { tail -30 gpurun_out/r5tp_t.txt; exit 3; }
tail -1 gpurun_out/r5tp_t.txt
for v in new old; do
  d=$GRAFT_REPO_ROOT; [ $v = old ] && d=$GRAFT_REPO_ROOT/ab_old
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/r5tp_$v
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5tp_$v -o run -- python3 $d/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1) || exit 6
  f=$(find gpurun_out/r5tp_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 - "$f" <<'PY'
import csv,sys
tot=0
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"])>1000:
        us=float(r["AverageNs"])/1000; n=int(r["Calls"])//1100
        tot+=us*n; print(f'{r["Name"][:58]:58s} {us:6.2f} x{n}')
print(f"kernel time per step {tot:.2f} us")
PY
done
for r in 1 2; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    a=$(cd $d && timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(cd $d && timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "$v 20/5 $a 2000/200 $b"
  done
done

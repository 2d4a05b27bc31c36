#!/bin/bash
# Multi-tenant packing curve: K independent sample-config jobs on one MI355X.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/pack.jsonl; : > $out
STEPS=${STEPS:-2000}
for mode in graph procs; do
  for K in 1 2 4 8; do
    if [ $K -eq 1 ]; then
      timeout -k 10 240 python bench.py --steps $STEPS --warmup 200 >> $out 2> gpurun_out/pack_err.log || exit 7
    else
      timeout -k 10 240 python bench.py --jobs $K --pack $mode --steps $STEPS --warmup 200 >> $out 2> gpurun_out/pack_err.log || exit 7
    fi
    tail -1 $out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', $K, d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# Packed (one process, one graph with K branches) curve, fused dense backward on and off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/pack2.jsonl; : > $out
for fd in 1 0; do
  for K in 1 2 4 8; do
    if [ $K -eq 1 ]; then
      CSA_FUSED_DENSE=$fd timeout -k 10 240 python bench.py --steps 2000 --warmup 200 >> $out 2> gpurun_out/pack_err.log || exit 7
    else
      CSA_FUSED_DENSE=$fd timeout -k 10 240 python bench.py --jobs $K --pack graph --steps 2000 --warmup 200 >> $out 2> gpurun_out/pack_err.log || exit 7
    fi
    tail -1 $out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused=$fd', $K, d['value'], d['ms_per_step'])"
  done
done

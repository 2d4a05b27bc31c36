#!/bin/bash
# Round 5: the pair backward loads bn_act_apply's forward BatchNorm tables instead of
# folding the statistic slab in every workgroup (CSA_PAIR_BN_TAB, default 1).  Numerics,
# per-block stamps, then the bench A/B, alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5tb_t.txt 2>&1 || { tail -30 gpurun_out/r5tb_t.txt; exit 3; }
tail -1 gpurun_out/r5tb_t.txt
for v in 1 0; do
  CSA_PAIR_BN_TAB=$v MB_HF=1 MB_CP_BLOCKS=1,350,699 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5tb_mb$v.txt 2>&1 || { tail -5 gpurun_out/r5tb_mb$v.txt; exit 4; }
  echo "tab=$v"; grep -E "HF:|pair alone block|updates block" gpurun_out/r5tb_mb$v.txt
done
for r in 1 2; do
  for v in 0 1; do
    a=$(CSA_PAIR_BN_TAB=$v timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(CSA_PAIR_BN_TAB=$v timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "tab=$v 20/5 $a 2000/200 $b"
  done
done

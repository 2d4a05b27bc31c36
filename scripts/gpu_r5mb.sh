#!/bin/bash
# Round 5: pair-backward route operands prefetched with the prologue — numerics, the
# block-0 phase stamps (MB_HF), bench in both shapes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5mb_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5mb_tests.log; [ $rc -ne 0 ] && exit $rc
MB_HF=1 timeout -k 10 200 python3 scripts/microbench.py --reps 200 > gpurun_out/r5mb.txt 2>&1 || { tail -20 gpurun_out/r5mb.txt; exit 3; }
grep -E "HF:|block 0" gpurun_out/r5mb.txt
for r in 1 2; do
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5mb_b20.json 2>> gpurun_out/r5mb.err || exit 4
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5mb_b2000.json 2>> gpurun_out/r5mb.err || exit 5
echo "bench 20/5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5mb_b20.json); 2000/200 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5mb_b2000.json)"
done
for w in 0 1; do
CSA_DU_WIDE=$w timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5mb_w$w.json 2>> gpurun_out/r5mb.err || exit 6
echo "du_wide=$w 2000/200 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5mb_w$w.json)"
done

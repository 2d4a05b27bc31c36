#!/bin/bash
# Deterministic lowerings + optimizer-carried dense updates (numerics, then A/B bench).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
# timeout -k 10 400 python3 -u -m pytest tests/test_deterministic.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4f_det.log 2>&1
# rc=$?; echo "det rc=$rc"; grep -E "passed|failed" gpurun_out/r4f_det.log | tail -3
# [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/r4f_det.log | tail -60; exit $rc; }
for c in split; do
CSA_DU_CARRIER=$c timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py -x -v -k "horizontal_fusion or run_steps_groups or optimizers_match" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4f_hf_$c.log 2>&1
rc=$?; echo "hfuse-$c rc=$rc"; grep -E "passed|failed" gpurun_out/r4f_hf_$c.log | tail -3
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/r4f_hf_$c.log | tail -60; exit $rc; }
done
for r in 1 2 3; do for c in pair split; do
CSA_DU_CARRIER=$c timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4f_b.json 2>> gpurun_out/r4f_bench.err || { tail -20 gpurun_out/r4f_bench.err; exit 4; }
echo "carrier=$c $(python3 -c "import json;d=json.load(open('gpurun_out/r4f_b.json'));print(d['ms_per_step'], d['value'])")"
done; done

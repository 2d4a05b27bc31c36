#!/bin/bash
# A/B: register budget (waves per SIMD) of the pair backward carrying the dense updates.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for o in 5 6; do CSA_HF_OCC=$o timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py -x -q -k "horizontal_fusion" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4l_t.log 2>&1 || { tail -30 gpurun_out/r4l_t.log; exit 3; }; done
echo tests ok
for o in 0 5 6; do CSA_HF_OCC=$o MB_HF=1 timeout -k 10 200 python scripts/microbench.py --reps 100 2>&1 | grep "HF:" | sed "s/^/occ=$o /"; done
b() {
env $1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4l_b.json 2>> gpurun_out/r4l.err || { tail -20 gpurun_out/r4l.err; exit 4; }
echo "$1 $(python3 -c "import json;d=json.load(open('gpurun_out/r4l_b.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2 3; do b CSA_HF_OCC=0; b CSA_HF_OCC=5; b CSA_HF_OCC=6; done

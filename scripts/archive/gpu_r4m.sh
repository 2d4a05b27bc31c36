#!/bin/bash
# Precomputed pair-backward index tables: numerics, block-0 stamps, A/B bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_hip_step.py -x -q -k "step_matches_torch and (sample or pair or relu_bias) or horizontal_fusion or run_steps or optimizers" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4m_t.log 2>&1 || { grep -E "passed|failed|Error" gpurun_out/r4m_t.log | tail -20; exit 3; }
grep -E "passed|failed" gpurun_out/r4m_t.log | tail -2
for t in 1 0; do CSA_CP_TABS=$t MB_HF=1 timeout -k 10 200 python scripts/microbench.py --reps 100 2>&1 | grep -E "HF:|block 0" | sed "s/^/tabs=$t /"; done
b() {
env $1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4m_b.json 2>> gpurun_out/r4m.err || { tail -20 gpurun_out/r4m.err; exit 4; }
echo "$1 $(python3 -c "import json;d=json.load(open('gpurun_out/r4m_b.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2 3; do b CSA_CP_TABS=0; b CSA_CP_TABS=1; done

#!/bin/bash
# fc2's deferred update carried by fc1's input-gradient launch: numerics, then A/B bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_hip_step.py -x -q -k "horizontal_fusion or run_steps or optimizers or step_matches_torch and (sample or deep20 or dense3_act or leaky)" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4s_t.log 2>&1 || { grep -E "passed|failed|Error|assert" gpurun_out/r4s_t.log | tail -20 | cut -c1-400; exit 3; }
grep -E "passed|failed" gpurun_out/r4s_t.log | tail -1
b() {
env $1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4s_b.json 2>> gpurun_out/r4s.err || { tail -20 gpurun_out/r4s.err; exit 4; }
echo "$1 $(python3 -c "import json;d=json.load(open('gpurun_out/r4s_b.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2 3; do b CSA_HF_DGRAD_CARRY=0; b CSA_HF_DGRAD_CARRY=1; done

#!/bin/bash
# DP soak (rehearsal: 2 ranks sharing the one GPU, xGMI collectives): 20k steps of the tuned
# program, every channel / tail health word checked (agreed over ranks) after the loop
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for s in allreduce:hf allreduce ps:hf lowrank; do
  CSA_DIST_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --strategy $s --steps 20000 --warmup 100 > gpurun_out/dpsoak_$s.json 2> gpurun_out/dpsoak_$s.err || { echo "$s failed"; grep -v "^\[Gloo\]" gpurun_out/dpsoak_$s.err | tail -20; exit 3; }
  python3 -c "
import json
line=[l for l in open('gpurun_out/dpsoak_$s.json') if l.startswith('{')][0]
d=json.loads(line); c=d['config']
print('$s', d['steps'], d['ms_per_step'], c['collectives'], d['final_loss'])
"
done

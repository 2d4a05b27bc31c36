#!/bin/bash
# Rehearsal of bench.py --gpus 8 on the one-GPU box (8 ranks time-slicing cuda:0; NOT a
# multi-GPU number): the world-8 code path end to end.  A progress line every 30 s.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
( for i in $(seq 1 40); do sleep 30; echo "$(date +%T) still running" >> gpurun_out/rehearse_8.progress; done ) &
ticker=$!
CSA_DIST_SHARED_GPU=1 timeout -k 10 1000 python3 bench.py --gpus 8 --steps 10 --warmup 3 > gpurun_out/rehearse_8.json 2> gpurun_out/rehearse_8.err
rc=$?
kill $ticker 2>/dev/null
grep -v "^\[Gloo\]" gpurun_out/rehearse_8.err | tail -5
python3 -c "
import json
line=[l for l in open('gpurun_out/rehearse_8.json') if l.startswith('{')][0]
d=json.loads(line); c=d['config']
print(d['n_gpus'], d['ms_per_step'], c['parallelism'], c['collectives'], c.get('strategy_tuning_ms_per_step'))
" || true
exit $rc

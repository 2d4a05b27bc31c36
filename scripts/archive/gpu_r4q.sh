#!/bin/bash
# Round-4 final measurements: smoke, bench (driver shape + long), packed K curve, kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4q_smoke.log 2>&1 || { tail -20 gpurun_out/r4q_smoke.log; exit 3; }
echo "smoke ok: $(tail -1 gpurun_out/r4q_smoke.log)"
for run in "20 5" "2000 200" "20 5" "2000 200"; do set -- $run
timeout -k 10 200 python bench.py --steps $1 --warmup $2 > gpurun_out/r4q_b_$1.json 2>> gpurun_out/r4q_bench.err || { tail -20 gpurun_out/r4q_bench.err; exit 4; }
echo "steps=$1 warmup=$2 $(cat gpurun_out/r4q_b_$1.json)"
done
for w in 400 100 400 100; do
CSA_WARM_MS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4q_w.json 2>> gpurun_out/r4q_bench.err || { tail -20 gpurun_out/r4q_bench.err; exit 4; }
echo "warm_ms=$w steps=20 $(python3 -c "import json;d=json.load(open('gpurun_out/r4q_w.json'));print(d['ms_per_step'], d['value'])")"
done
for k in 2 4 8; do
timeout -k 10 200 python bench.py --jobs $k --pack graph --steps 2000 --warmup 200 > gpurun_out/r4q_pack$k.json 2>> gpurun_out/r4q_bench.err || { tail -20 gpurun_out/r4q_bench.err; exit 5; }
echo "pack K=$k $(python3 -c "import json;d=json.load(open('gpurun_out/r4q_pack$k.json'));print(d['ms_per_step'], d['value'])")"
done
rm -rf $R/gpurun_out/trace; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace --steps 1100 > gpurun_out/r4q_trace.md && head -14 gpurun_out/r4q_trace.md

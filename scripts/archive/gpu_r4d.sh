#!/bin/bash
# Round-4 measurements: 1-GPU bench (driver shape + long), packed K = 1/2/4/8, kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for run in "20 5" "2000 200" "20 5" "2000 200"; do set -- $run
timeout -k 10 200 python bench.py --steps $1 --warmup $2 > gpurun_out/r4d_b.json 2>> gpurun_out/r4d_bench.err || { tail -20 gpurun_out/r4d_bench.err; exit 4; }
echo "steps=$1 warmup=$2 $(python3 -c "import json;d=json.load(open('gpurun_out/r4d_b.json'));print(d['ms_per_step'], d['value'])")"
done
for k in 1 2 4 8; do
timeout -k 10 200 python bench.py --jobs $k --pack graph --steps 2000 --warmup 200 > gpurun_out/r4d_pack$k.json 2>> gpurun_out/r4d_bench.err || { tail -20 gpurun_out/r4d_bench.err; exit 5; }
echo "pack K=$k $(python3 -c "import json;d=json.load(open('gpurun_out/r4d_pack$k.json'));print(d['ms_per_step'], d['value'])")"
done
for b in 100 200 400; do
timeout -k 10 200 python bench.py --batch $b --steps 400 --warmup 100 > gpurun_out/r4d_batch$b.json 2>> gpurun_out/r4d_bench.err || { tail -20 gpurun_out/r4d_bench.err; exit 7; }
echo "batch=$b $(python3 -c "import json;d=json.load(open('gpurun_out/r4d_batch$b.json'));print(d['ms_per_step'], d['value'])")"
done
rm -rf $R/gpurun_out/trace; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace --steps 1100 > gpurun_out/r4d_trace.md && cat gpurun_out/r4d_trace.md

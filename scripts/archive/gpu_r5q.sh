#!/bin/bash
# Round 5 rehearsal: the whole GPU suite, smoke(), the driver's bench shape, step traces
# (1-GPU program and the DP ":hf" program at world 1).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/r5q_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/r5q_tests.log | tail -5 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5q_smoke.txt 2>&1 || { tail -20 gpurun_out/r5q_smoke.txt; exit 3; }
tail -1 gpurun_out/r5q_smoke.txt
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5q_b20.json 2>> gpurun_out/r5q.err || exit 4
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5q_b2000.json 2>> gpurun_out/r5q.err || exit 5
echo "bench 20/5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5q_b20.json); 2000/200 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5q_b2000.json)"
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5q_tr1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 6
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5q_trdp -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_dp1.py --strategy allreduce:hf --xgmi 0 --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 7
cd $GRAFT_REPO_ROOT
python3 scripts/step_timeline.py $(find gpurun_out/r5q_tr1 -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 2 > gpurun_out/r5q_tl1.txt
python3 scripts/step_timeline.py $(find gpurun_out/r5q_trdp -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 2 > gpurun_out/r5q_tldp.txt
cat gpurun_out/r5q_tl1.txt

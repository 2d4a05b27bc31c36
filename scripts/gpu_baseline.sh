#!/bin/bash
# First GPU measurement: torch-op engine (graph and eager) + rocprofv3 kernel stats.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --backend torch --steps 500 --warmup 50 > gpurun_out/bench_torch_graph.json 2> gpurun_out/bench_torch_graph.err
timeout -k 10 300 python bench.py --backend torch --steps 200 --warmup 20 --no-graph > gpurun_out/bench_torch_eager.json 2> gpurun_out/bench_torch_eager.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_torch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --backend torch --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_torch.log" 2>&1
cat "$GRAFT_REPO_ROOT"/gpurun_out/bench_torch_*.json

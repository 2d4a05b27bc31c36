#!/bin/bash
# round 6: fixed cost of the short timed loop (bench 20/5 vs 2000/200): host launch,
# device time, synchronize wake-up — default runtime vs spin scheduling vs runtime knobs
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_default.json 2>gpurun_out/lo.err || exit $?
MB_SPIN=1 $T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_spin.json 2>>gpurun_out/lo.err || exit $?
ROC_ACTIVE_WAIT_TIMEOUT=5000 $T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_active.json 2>>gpurun_out/lo.err || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_pc0.json 2>>gpurun_out/lo.err || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 $T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_pc1.json 2>>gpurun_out/lo.err || exit $?
MB_K=200 $T 120 python scripts/mb/launch_overhead.py > gpurun_out/lo_k200.json 2>>gpurun_out/lo.err || exit $?
$T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/b20.json 2>>gpurun_out/lo.err || exit $?
cat gpurun_out/lo_*.json gpurun_out/b20.json

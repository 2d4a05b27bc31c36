#!/bin/bash
# Rehearsal of the driver's N-GPU bench path on a one-GPU box: bench.py --gpus N starts
# torch.distributed.run itself; CSA_DIST_SHARED_GPU=1 puts every rank on cuda:0 over gloo
# with the xGMI peer-buffer collectives (strategy tuner, HIP programs, timed loop, JSON).
# The ms/step of ranks time-slicing one GPU is NOT a multi-GPU number.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for n in 2 4; do
  CSA_DIST_SHARED_GPU=1 timeout -k 10 500 python3 bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { echo "gpus $n failed rc=$?"; tail -30 gpurun_out/rehearse_$n.err; exit 3; }
  echo "gpus $n: $(cat gpurun_out/rehearse_$n.json | cut -c1-400)"
done

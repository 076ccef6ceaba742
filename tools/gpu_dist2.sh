#!/bin/bash
# Rehearsal of the pipelined multi-rank bench: 2 and 3 ranks on one GPU, host-callback communicator.
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2952$w bench.py --gpus $w --comm host --steps 4 --warmup 1 --cpu-baseline off > gpurun_out/dist_${tag}_w$w.log 2>&1 || { echo FAILED w$w; tail -20 gpurun_out/dist_${tag}_w$w.log; exit 1; }
  grep metric gpurun_out/dist_${tag}_w$w.log | cut -c1-700
done

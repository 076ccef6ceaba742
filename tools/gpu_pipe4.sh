#!/bin/bash
# 16384 with the 32-CU reservation, 8192 c24, and the pipelined dist path at world size 1 (RCCL).
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, n, args...
  local nm=$1 n=$2; shift 2
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/pipe_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/pipe_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'])" gpurun_out/pipe_${tag}_$nm.log $nm
}


timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --force-dist --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pipe_${tag}_dist1.log 2>&1 || { echo FAILED dist1; tail -20 gpurun_out/pipe_${tag}_dist1.log; exit 1; }
grep metric gpurun_out/pipe_${tag}_dist1.log | cut -c1-900

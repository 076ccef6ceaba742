#!/bin/bash
# Pipelined lanes on one GPU (stage-1 panel factors of one lane beside the other's updates).
tag=${1:-dev}; n=${2:-8192}; k=${3:-8}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/lanes_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/lanes_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'])" gpurun_out/lanes_${tag}_$nm.log $nm
}
run L2 --lanes 2 --steps $k --warmup 2 || exit 1
BRD_S1_TARGET=192 run L2_t192 --lanes 2 --steps $k --warmup 2 || exit 1
run L3 --lanes 3 --steps $k --warmup 3 || exit 1
BRD_S1_TARGET=160 run L3_t160 --lanes 3 --steps $k --warmup 3 || exit 1

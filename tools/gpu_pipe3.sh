#!/bin/bash
# Reproducibility of the c64 sweet spot; apply target under overlap.
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, n, args...
  local nm=$1 n=$2; shift 2
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/pipe_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/pipe_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'])" gpurun_out/pipe_${tag}_$nm.log $nm
}
run c64a 8192 --pipeline on --s2-cus 64 --steps 8 --warmup 2 || exit 1
run c32 8192 --pipeline on --s2-cus 32 --steps 8 --warmup 2 || exit 1
BRD_S1_TARGET=256 run c64_t256 8192 --pipeline on --s2-cus 64 --steps 8 --warmup 2 || exit 1
BRD_S1_TARGET=224 run c64_t224 8192 --pipeline on --s2-cus 64 --steps 8 --warmup 2 || exit 1
BRD_S1_TARGET=160 run c64_t160 8192 --pipeline on --s2-cus 64 --steps 8 --warmup 2 || exit 1
run c64b 8192 --pipeline on --s2-cus 64 --steps 8 --warmup 2 || exit 1

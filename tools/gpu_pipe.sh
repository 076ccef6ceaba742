#!/bin/bash
# Pipelined-stream experiment: serial vs pipelined bench lines, stage-2 CU reservations.
# usage: bash tools/gpu_pipe.sh <tag> [n] [steps]
tag=${1:-dev}; n=${2:-8192}; k=${3:-6}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/pipe_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/pipe_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['roofline']['achieved'], d['kernel_ms_per_step'])" gpurun_out/pipe_${tag}_$nm.log $nm
}
run off --pipeline off --steps 3 --warmup 1 || exit 1
BRD_S1_SPW_SEARCH=0 true
for c in 64 40 96; do run on_c$c --pipeline on --s2-cus $c --steps $k --warmup 2 || exit 1; done

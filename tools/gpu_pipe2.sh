#!/bin/bash
# CU-reservation sweep for the pipelined bench (8192), and stage-2 grid sizes at 16384.
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, n, args...
  local nm=$1 n=$2; shift 2
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/pipe_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/pipe_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'])" gpurun_out/pipe_${tag}_$nm.log $nm
}
for c in 48 56 72 80 128; do run on8k_c$c 8192 --pipeline on --s2-cus $c --steps 8 --warmup 2 || exit 1; done
for g in 64 128; do BRD_S2_GRID=$g run off16k_g$g 16384 --pipeline off --steps 2 --warmup 1 || exit 1; done
for c in 64 128; do run on16k_c$c 16384 --pipeline on --s2-cus $c --steps 4 --warmup 1 || exit 1; done

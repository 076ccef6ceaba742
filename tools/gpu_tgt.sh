#!/bin/bash
# Stage-1 apply target beside a 32-CU stage 2 (pipelined, N = 8192, 8 steps).
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --cpu-baseline off --one-at-a-time off "$@" > gpurun_out/tgt_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/tgt_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'])" gpurun_out/tgt_${tag}_$nm.log $nm
}
run t224 --steps 8 --warmup 2 || exit 1
for t in 216 208 192 240; do BRD_S1_TARGET=$t run t$t --steps 8 --warmup 2 || exit 1; done

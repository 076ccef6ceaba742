#!/bin/bash
# Leading-dimension padding: serial and pipelined bench lines with lda = n and n + pad.
tag=${1:-dev}; n=${2:-8192}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --n $n --cpu-baseline off "$@" > gpurun_out/pad_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/pad_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'], d['roofline']['achieved'])" gpurun_out/pad_${tag}_$nm.log $nm
}
run off_p0 --pipeline off --steps 3 --warmup 1 || exit 1
run off_p256 --pipeline off --pad 256 --steps 3 --warmup 1 || exit 1
run off_p32 --pipeline off --pad 32 --steps 3 --warmup 1 || exit 1
run on_p256 --pad 256 --steps 8 --warmup 2 || exit 1

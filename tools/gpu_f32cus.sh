#!/bin/bash
# fp32 pipelined: stage-2 CU reservation (stage 1 is the longer stage there).
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 32 24 16; do
  timeout -k 10 300 python bench.py --dtype f32 --s2-cus $c --steps 8 --cpu-baseline off --one-at-a-time off > gpurun_out/f32c_${tag}_$c.log 2>&1 || { echo FAILED $c; tail -5 gpurun_out/f32c_${tag}_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'])" gpurun_out/f32c_${tag}_$c.log c$c
done

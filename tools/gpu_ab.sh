#!/bin/bash
# Parity tests (stage 1 + dist) then serial and pipelined bench lines.
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$tag.log 2>&1 || { echo TESTS FAILED; tail -15 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/ab_${tag}_$nm.log 2>&1 || { echo FAILED $nm; tail -5 gpurun_out/ab_${tag}_$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms_per_step'], d['roofline']['achieved'], d.get('one_at_a_time'))" gpurun_out/ab_${tag}_$nm.log $nm
}
run f64 || exit 1
run f32 --dtype f32 --one-at-a-time on || exit 1

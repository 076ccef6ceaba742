#!/bin/bash
# Bench lines for the other BASELINE configs (fp32 8192, fp64 16384), pipelined + one at a time.
tag=${1:-dev}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dtype f32 --cpu-baseline off > gpurun_out/b_${tag}_f32.log 2>&1 || { echo FAILED f32; tail -5 gpurun_out/b_${tag}_f32.log; exit 1; }
grep metric gpurun_out/b_${tag}_f32.log | cut -c1-300
timeout -k 10 500 python bench.py --n 16384 --cpu-baseline off > gpurun_out/b_${tag}_16k.log 2>&1 || { echo FAILED 16k; tail -5 gpurun_out/b_${tag}_16k.log; exit 1; }
grep metric gpurun_out/b_${tag}_16k.log | cut -c1-300

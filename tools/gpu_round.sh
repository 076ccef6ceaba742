#!/bin/bash
# One GPU session: all -m gpu tests, smoke(), a default bench line, a rocprofv3 kernel trace.
# usage: bash tools/gpu_round.sh <tag> [n]
tag=${1:-dev}; n=${2:-8192}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$tag.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/t_$tag.log | tail -8
[ $rc -ne 0 ] && exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_$tag.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/s_$tag.log; exit 1; }
tail -1 gpurun_out/s_$tag.log
timeout -k 10 400 python bench.py --n $n > gpurun_out/b_$tag.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/b_$tag.log; exit 1; }
grep metric gpurun_out/b_$tag.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --n $n --steps 2 --warmup 1 --cpu-baseline off --one-at-a-time off > gpurun_out/p_$tag.log 2>&1 || { echo PROF FAILED; exit 1; }
grep metric gpurun_out/p_$tag.log
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1); echo "stats: $f"; cut -c1-160 "$f" | head -12

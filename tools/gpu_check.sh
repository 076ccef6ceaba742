#!/bin/bash
# One GPU session: parity tests, a bench line, and a rocprofv3 kernel trace.
# usage: bash tools/gpu_check.sh <tag> [n]
tag=${1:-dev}; n=${2:-8192}
cd $GRAFT_REPO_ROOT
make -s -C oracle liboracle.so >/dev/null || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/t_$tag.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed|Error" gpurun_out/t_$tag.log | tail -5
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py --n $n --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/b_$tag.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/b_$tag.log; exit 1; }
grep metric gpurun_out/b_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'stage',d['stage_ms'],'k',d['kernel_ms_per_step'],'roof',d['roofline']['achieved'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --n $n --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/p_$tag.log 2>&1 || { echo PROF FAILED; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1); echo "stats: $f"; cut -c1-160 "$f" | head -12

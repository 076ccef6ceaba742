#!/bin/bash
# Stage-2 GPU check: parity tests of stage 2 + the stamped timeline harness + bench line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "stage2 or two_stage" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/t2.log; [ $rc -ne 0 ] && exit 1
timeout -k 5 60 ./tools/s2bench ${1:-8192} > gpurun_out/s2b.log 2>&1 || { echo S2BENCH FAILED; tail gpurun_out/s2b.log; exit 1; }
cat gpurun_out/s2b.log
timeout -k 10 300 python bench.py --n 8192 --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/b2.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/b2.log; exit 1; }
grep metric gpurun_out/b2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'stage',d['stage_ms'],'k',d['kernel_ms_per_step'])"

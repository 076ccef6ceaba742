#!/bin/bash
# Stage-1 GPU check: stage-1 parity tests, kernel stamps, stage-1 timing.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "stage1 or two_stage" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/t1.log; [ $rc -ne 0 ] && exit 1
timeout -k 5 60 ./tools/kbench 8192 > gpurun_out/kb.log 2>&1 || { echo KBENCH FAILED; tail gpurun_out/kb.log; exit 1; }
grep -E "level=0 groups=16" gpurun_out/kb.log | tail -2
rm -f /tmp/s1time_ref.npy
timeout -k 5 120 python tools/s1time.py 8192 default 2>&1 | tail -1

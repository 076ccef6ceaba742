cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
BRD_BLK_RPX=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_parity.py -k "blocked or structured or extreme or fixture or gen1024" > gpurun_out/rpx_tests.log 2>&1 || { echo "FAIL tests"; tail -30 gpurun_out/rpx_tests.log; exit 1; }
tail -1 gpurun_out/rpx_tests.log
bash tools/blk_ab.sh rpx "BRD_BLK_RPX=1;BRD_BLK_RPX=2;BRD_BLK_RPX=3"

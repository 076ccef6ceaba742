cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/blk_check.py check > gpurun_out/blk7.log 2>&1 && \
BRD_S1_STAMPS=1 timeout -k 10 300 python -u tools/blk_check.py t8 > gpurun_out/blk7s.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_blk7 -o run -- python3 tools/blk_check.py t8 > gpurun_out/blk7p.log 2>&1
echo rc=$?
cat gpurun_out/blk7.log gpurun_out/blk7s.log | grep -v amdgpu.ids | tail -12
f=$(find gpurun_out/prof_blk7 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep blk

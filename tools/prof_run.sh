cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2048 -o run -- python3 bench.py --n 2048 --steps 1 --warmup 1 --cpu-baseline off > gpurun_out/prof2048.log 2>&1
echo EXIT $?
find gpurun_out/prof2048 -name "*stats*" | head

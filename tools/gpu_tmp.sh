cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
E="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29511"
A="--steps,12,--warmup,3,--force-dist"
bash tools/bench_ab.sh "dist8|$E|$A" "dist0|$E BRD_RCCL_MAX_CTAS=0|$A"

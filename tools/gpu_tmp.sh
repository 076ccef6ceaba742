cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_session.sh ab3 "s2:8192:BASE=1;BRD_LIB=tools/reflib/old.so" || exit 1
bash tools/bench_ab.sh "cur||--steps,20,--warmup,5" "old|BRD_LIB=tools/reflib/old.so|--steps,20,--warmup,5"

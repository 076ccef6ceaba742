# one-reduction-at-a-time A/B of the upper-level apply run floor (developer tool)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps,12,--warmup,3,--pipeline,off"
bash tools/bench_ab.sh "m1||$A" "m2|BRD_S1_MINRUN1=2|$A" "m3|BRD_S1_MINRUN1=3|$A" "m1b||$A" "m2b|BRD_S1_MINRUN1=2|$A"

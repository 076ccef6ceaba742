cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps,16,--warmup,4,--one-at-a-time,off"
bash tools/bench_ab.sh "base||$A" "m1_4|BRD_S1_MINRUN1=4|$A" "m1_8|BRD_S1_MINRUN1=8|$A" "m0_3|BRD_S1_MINRUN0=3|$A" "m0_3m1_4|BRD_S1_MINRUN0=3 BRD_S1_MINRUN1=4|$A" "m1_16|BRD_S1_MINRUN1=16|$A" "base2||$A"

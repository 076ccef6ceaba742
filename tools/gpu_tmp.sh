cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps,16,--warmup,4,--one-at-a-time,off"
bash tools/bench_ab.sh "base||$A" "t112|BRD_S1_TARGET=112|$A" "t160|BRD_S1_TARGET=160|$A" "t192|BRD_S1_TARGET=192|$A" "t128|BRD_S1_TARGET=128|$A" "base2||$A" "r0|BRD_S2_RAMP=0|$A"

# one-reduction-at-a-time A/B (developer tool): bash tools/minrun_ab.sh "label|ENV" ...
# (default: the upper-level apply run floor, BRD_S1_MINRUN1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps,12,--warmup,3,--pipeline,off"
if [ $# -eq 0 ]; then set -- "m1|" "m2|BRD_S1_MINRUN1=2" "m3|BRD_S1_MINRUN1=3"; fi
specs=()
for s in "$@"; do specs+=("$s|$A"); done
bash tools/bench_ab.sh "${specs[@]}"

# final measurement session of a round (developer tool): bench lines + rocprof stats per config
cd $GRAFT_REPO_ROOT && bash tools/gpu_session.sh ${1:-fin} bench prof bench:--dtype,f32 prof:8192:f32 bench:--n,16384 prof:16384:f64

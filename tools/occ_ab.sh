# fp32 stage-1 apply occupancy A/B (developer tool): two workgroups per CU in the
# stream (default) vs the one-per-CU variants (BRD_S1_OCC2=0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "overlap or reduce_many" > gpurun_out/t_occ.log 2>&1; echo "PYTEST rc=$?"; tail -1 gpurun_out/t_occ.log
A="--dtype,f32,--steps,20,--warmup,5"
bash tools/bench_ab.sh "new||$A" "old|BRD_S1_OCC2=0|$A" "new2||$A" "old2|BRD_S1_OCC2=0|$A"

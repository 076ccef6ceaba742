# A/B of the number of lanes (developer tool): the stream bench on one GPU,
# then the distributed path at world size 1 over RCCL (--force-dist).
#   bash tools/lanes_ab.sh "4 8 4 8" "4 8"
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${1:-4 8 4 8}; do
  timeout -k 10 300 python bench.py --cpu-baseline off --one-at-a-time off --lanes $v > gpurun_out/ln_$v.log 2>&1 || exit 1
  grep metric gpurun_out/ln_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $v', d['value'], d['ms_per_step'], d['stage_ms'])"
done
for v in ${2:-4 8}; do
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 \
    timeout -k 10 300 python bench.py --cpu-baseline off --force-dist --steps 12 --warmup 2 --lanes $v > gpurun_out/lnd_$v.log 2>&1 || exit 1
  grep metric gpurun_out/lnd_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dist lanes $v', d['value'], d['ms_per_step'], d['stage_ms'])"
done

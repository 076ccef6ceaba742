cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for cfg in "8 32" "12 20" "16 16" "10 24" "8 24"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --lanes $1 --s2-cus $2 --steps 24 --warmup 4 --one-at-a-time off --cpu-baseline off > gpurun_out/lanes_$1_$2.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/lanes_$1_$2.log; exit 1; }
  echo "lanes $1 s2_cus $2: $(grep -o '"value": [0-9.]*' gpurun_out/lanes_$1_$2.log | head -1)"
done

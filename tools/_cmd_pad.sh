cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for pad in 0 32 256; do
  timeout -k 10 300 python bench.py --pipeline off --steps 5 --warmup 2 --pad $pad --cpu-baseline off > gpurun_out/pad_$pad.log 2>&1 || { echo "FAIL $pad"; tail -3 gpurun_out/pad_$pad.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/pad_$pad.log').read().strip().splitlines()[-1])
print('pad $pad', d['value'], d['stage_ms'], d['kernel_ms_per_step'])
"
done

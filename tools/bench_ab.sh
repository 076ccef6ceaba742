# Bench A/B (developer tool): bash tools/bench_ab.sh "<label>|<env>|<bench args, comma-separated>" ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r lab envs args <<< "$spec"
  env $envs timeout -k 10 300 python bench.py ${args//,/ } --cpu-baseline off > gpurun_out/ab_$lab.log 2>&1 || { echo "$lab FAILED"; tail -3 gpurun_out/ab_$lab.log; exit 1; }
  grep metric gpurun_out/ab_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d.get('one_at_a_time') or {}; print('$lab', d['value'], d['ms_per_step'], d['stage_ms'], o.get('ms_per_step'), o.get('stage_ms'), d['roofline']['frac'], d.get('kernel_ms_per_step'))"
done

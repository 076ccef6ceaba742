#!/bin/bash
# Blocked stage-1 A/B (developer tool): for each ';'-separated environment
# variant, the stage-1 timing of tools/blk_check.py t8 and a rocprofv3
# kernel-stats pass of the same run (per-kernel averages of the blocked path).
#   bash tools/blk_ab.sh TAG "A=1;A=2" [check]
tag=$1; vars=$2; chk=$3
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "$chk" = "check" ]; then
  timeout -k 10 300 python -u tools/blk_check.py check > gpurun_out/blkab_${tag}_check.log 2>&1 || { echo CHECK FAILED; tail -5 gpurun_out/blkab_${tag}_check.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/blkab_${tag}_check.log
fi
IFS=';' read -ra VS <<< "$vars"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  for kv in $v; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blkab_${tag}_$i -o run -- python3 tools/blk_check.py t8 > gpurun_out/blkab_${tag}_$i.log 2>&1 || { echo "RUN FAILED ($v)"; tail -5 gpurun_out/blkab_${tag}_$i.log; exit 1; }
  for kv in $v; do unset "${kv%%=*}"; done
  echo "== $v: $(grep timing gpurun_out/blkab_${tag}_$i.log)"; grep "phases" gpurun_out/blkab_${tag}_$i.log | tail -1
  f=$(find gpurun_out/blkab_${tag}_$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "blk::" in n:
        calls = int(r["Calls"]); tot = float(r["TotalDurationNs"]) / 1e6
        print(f"   {n.split('blk::')[1].split('(')[0]:28s} calls/run {calls/4:6.0f}  ms/run {tot/4:7.2f}  avg_us {tot*1e3/calls:8.1f}")
PY
done
echo SESSION OK

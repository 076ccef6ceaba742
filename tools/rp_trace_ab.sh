#!/bin/bash
# Read-pass kernel traces of library variants (developer tool):
#   bash tools/rp_trace_ab.sh LABEL[=LIB[=ARGS]] ...  (LIB empty: the in-tree build;
#   ARGS: extra bench.py flags, comma-separated)
# one rocprofv3 --kernel-trace run of a one-at-a-time bench step per variant,
# then tools/rp_curve.py prints the per-panel read-pass durations side by side.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
dirs=""
for spec in "$@"; do
  IFS='=' read -r lab lib args <<< "$spec"
  d=gpurun_out/rpt_$lab
  BRD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --steps 1 --warmup 1 --pipeline off --cpu-baseline off ${args//,/ } > $d.log 2>&1 || { echo "$lab FAILED"; tail -3 $d.log; exit 1; }
  dirs="$dirs $lab=$d"
done
python3 tools/rp_curve.py $dirs

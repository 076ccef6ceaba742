#!/bin/bash
# Stage-1 A/B timing of environment variants in one box session (developer tool).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f /tmp/s1time_ref.npy
n=${1:-8192}; shift
for v in "$@"; do
  env $v timeout -k 5 120 python tools/s1time.py $n "$v" 2>&1 | tail -1 || exit 1
done

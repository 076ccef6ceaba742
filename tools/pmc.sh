#!/bin/bash
# HBM traffic of the stage-1/stage-2 kernels from rocprofv3 PMC counters: one
# pass per counter (FETCH_SIZE, WRITE_SIZE), then per-kernel averages.
# usage: bash tools/pmc.sh <tag> [n] [dtype] [extra bench args, comma-separated]
# The summary (copied to profiles/rNN_pmc_n{n}_{dtype}.txt) is what bench.py's
# roofline.traffic reads for that configuration.
tag=${1:-dev}; n=${2:-8192}; dt=${3:-f64}; extra=${4:-}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${tag}_n${n}_${dt}_$c -o run -- python3 bench.py --n $n --dtype $dt --steps 1 --warmup 1 --cpu-baseline off --pipeline off ${extra//,/ } > gpurun_out/pmc_${tag}_n${n}_${dt}_$c.log 2>&1 || { echo "PMC $c FAILED"; tail -5 gpurun_out/pmc_${tag}_n${n}_${dt}_$c.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_n${n}_${dt}_FETCH_SIZE gpurun_out/pmc_${tag}_n${n}_${dt}_WRITE_SIZE | tee gpurun_out/pmc_${tag}_n${n}_${dt}.txt

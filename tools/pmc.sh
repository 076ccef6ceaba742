#!/bin/bash
# HBM traffic and MFMA utilisation of the stage-1/stage-2 kernels from
# rocprofv3 PMC counters: one pass per counter group (FETCH_SIZE; WRITE_SIZE;
# the MFMA group SQ_INSTS_VALU_MFMA_MOPS_F64/_F32 + SQ_VALU_MFMA_BUSY_CYCLES +
# GRBM_GUI_ACTIVE), then per-kernel averages.
# usage: bash tools/pmc.sh <tag> [n] [dtype] [extra bench args, comma-separated]
# The summary (copied to profiles/rNN_pmc_n{n}_{dtype}.txt) is what bench.py's
# roofline.traffic / mfma_util_counter read for that configuration.
tag=${1:-dev}; n=${2:-8192}; dt=${3:-f64}; extra=${4:-}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "$dt" = "f64" ]; then mops=SQ_INSTS_VALU_MFMA_MOPS_F64; else mops=SQ_INSTS_VALU_MFMA_MOPS_F32; fi
i=0
for c in FETCH_SIZE WRITE_SIZE "$mops SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${tag}_n${n}_${dt}_p$i -o run -- python3 bench.py --n $n --dtype $dt --steps 1 --warmup ${PMC_WARMUP:-1} --cpu-baseline off --pipeline off ${extra//,/ } > gpurun_out/pmc_${tag}_n${n}_${dt}_p$i.log 2>&1 || { echo "PMC pass $i ($c) FAILED"; tail -5 gpurun_out/pmc_${tag}_n${n}_${dt}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_n${n}_${dt}_p1 gpurun_out/pmc_${tag}_n${n}_${dt}_p2 gpurun_out/pmc_${tag}_n${n}_${dt}_p3 $dt | tee gpurun_out/pmc_${tag}_n${n}_${dt}.txt

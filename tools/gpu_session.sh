#!/bin/bash
# One gpurun session, built from steps (developer tool; replaces the round-1
# one-off gpu_*.sh scripts).  Every GPU step has its own time limit; the
# session stops at the first failing step.
#   bash tools/gpu_session.sh <tag> step [step ...]
# steps:
#   tests            all -m gpu tests (pytest, per-test timeouts)
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     one bench.py line (ARGS: comma-separated extra flags, e.g. bench:--dtype,f32)
#   prof[:N:DT:ARGS] rocprofv3 --kernel-trace --stats of a short bench (default one reduction at a time)
#   pmc[:N:DT:ARGS]  FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh) at N, dtype DT (+ bench args)
#   s1[:N]           stage-1 timing (tools/s1time.py)
#   s2[:N:VARS]      stage-2 timing per environment variant (VARS: ';'-separated, each 'K=V K2=V2')
#   py:FILE[:ARGS]   run a python file with comma-separated args
tag=$1; shift
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for st in "$@"; do
  name=${st%%:*}; arg=${st#*:}; [ "$arg" = "$st" ] && arg=""
  case $name in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/t_$tag.log 2>&1; rc=$?
      echo "PYTEST rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/t_$tag.log | tail -8
      [ $rc -ne 0 ] && exit 1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_$tag.log 2>&1 \
        || { echo SMOKE FAILED; tail -5 gpurun_out/s_$tag.log; exit 1; }
      tail -1 gpurun_out/s_$tag.log ;;
    bench)
      a=${arg//,/ }; k=$(echo "$a" | tr -cd 'a-z0-9' | cut -c1-24)
      timeout -k 10 600 python bench.py $a > gpurun_out/b_${tag}_$k.log 2>&1 \
        || { echo BENCH FAILED; tail -5 gpurun_out/b_${tag}_$k.log; exit 1; }
      grep metric gpurun_out/b_${tag}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['stage_ms'], d.get('one_at_a_time'), d['kernel_ms_per_step'], d['roofline']['frac'])" ;;
    prof)
      # prof[:N[:DT[:ARGS]]]: default ARGS --pipeline,off (one reduction at a
      # time: the pass bench.py's roofline durations come from)
      n=$(echo "$arg" | cut -d: -f1); dt=$(echo "$arg" | cut -s -d: -f2); pa=$(echo "$arg" | cut -s -d: -f3)
      n=${n:-8192}; dt=${dt:-f64}; pa=${pa:---pipeline,off}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_${n}_$dt -o run -- \
        python3 bench.py --n $n --dtype $dt --steps 3 --warmup 1 --cpu-baseline off ${pa//,/ } > gpurun_out/p_${tag}_${n}_$dt.log 2>&1 \
        || { echo PROF FAILED; tail -5 gpurun_out/p_${tag}_${n}_$dt.log; exit 1; }
      grep metric gpurun_out/p_${tag}_${n}_$dt.log | cut -c1-400
      f=$(find gpurun_out/prof_${tag}_${n}_$dt -name "*kernel_stats.csv" | head -1); echo "stats: $f"; cut -c1-150 "$f" | head -10 ;;
    pmc)
      n=$(echo $arg | cut -d: -f1); dt=$(echo $arg | cut -s -d: -f2); ex=$(echo $arg | cut -s -d: -f3); bash tools/pmc.sh ${tag} ${n:-8192} ${dt:-f64} "$ex" || exit 1 ;;
    s1)
      # s1[:N[:VARS[:DT]]]: stage-1 timing per environment variant (';'-separated)
      n=$(echo "$arg" | cut -d: -f1); vars=$(echo "$arg" | cut -s -d: -f2); dt=$(echo "$arg" | cut -s -d: -f3)
      [ -z "$vars" ] && vars="BASE=1"
      IFS=';' read -ra VS <<< "$vars"
      for v in "${VS[@]}"; do
        env $v timeout -k 5 200 python tools/s1time.py ${n:-8192} "$v" ${dt:-f64} 2>&1 | tail -1 || exit 1
      done ;;
    s2)
      # s2[:N[:VARS[:DT]]]
      n=$(echo "$arg" | cut -d: -f1); vars=$(echo "$arg" | cut -s -d: -f2); dt=$(echo "$arg" | cut -s -d: -f3)
      [ -z "$vars" ] && vars="BASE=1"
      rm -f /tmp/s2time_ref.npy
      IFS=';' read -ra VS <<< "$vars"
      for v in "${VS[@]}"; do
        env $v timeout -k 5 200 python tools/s2time.py ${n:-8192} "$v" ${dt:-f64} 2>&1 | tail -1 || exit 1
      done ;;
    py)
      f=${arg%%:*}; a=${arg#*:}; [ "$a" = "$arg" ] && a=""
      timeout -k 10 600 python -u $f ${a//,/ } > gpurun_out/py_${tag}_$(basename $f .py).log 2>&1; rc=$?
      tail -30 gpurun_out/py_${tag}_$(basename $f .py).log; [ $rc -ne 0 ] && exit 1 ;;
    *) echo "unknown step $name"; exit 1 ;;
  esac
done
echo SESSION OK

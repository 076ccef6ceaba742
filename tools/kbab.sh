# A/B of the stage-1 apply micro-benchmark (developer tool):
#   bash tools/kbab.sh "<label>=<env> ..." [dtypes] [lds] [binary=kbench_ns]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; o=gpurun_out/kbab_${4:-kbench_ns}.log; : > $o
for dt in ${2:-f64 f32}; do for ld in ${3:-8192}; do for v in $1; do
  echo "== ${v%%=*} $dt ld=$ld" >> $o
  env ${v#*=} timeout -k 5 60 tools/${4:-kbench_ns} 8192 $dt 256 8160 $ld >> $o 2>&1 || exit 1
done; done; done
python3 - $o <<'PY'
import re, sys
cur=None
for line in open(sys.argv[1]):
    if line.startswith('=='): cur=line.strip(); vals={0:[],1:[]}; continue
    m='apply' in line and re.search(r'trans=(\d).*?: ([\d.]+) us',line)
    if m:
        vals[int(m.group(1))].append(float(m.group(2)))
        if len(vals[1])==4: print(cur, 'trans0 %.1f us  trans1 %.1f us'%(sorted(vals[0])[1],sorted(vals[1])[1]))
PY

cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in svdsolver_amd/lib/libbrd_hip.so tools/diaglib/d_p1.so tools/diaglib/d_p2.so tools/diaglib/d_q1a.so tools/diaglib/d_q1b.so; do
  t=$(basename $lib .so)
  BRD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dg_$t -o run -- python3 tools/rp_diag.py > gpurun_out/dg_$t.log 2>&1 || { echo "FAIL $t"; tail -3 gpurun_out/dg_$t.log; exit 1; }
  f=$(find gpurun_out/dg_$t -name "*kernel_stats.csv" | head -1)
  echo "== $t"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('prep', 'cqr_q1', 'cqr_gram', 'cqr_v')): print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done

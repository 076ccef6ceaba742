cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in svdsolver_amd/lib/libbrd_hip.so tools/diaglib/nob.so tools/diaglib/nobnom.so; do
  t=$(basename $lib .so)
  BRD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/diag_$t -o run -- python3 tools/rp_diag.py > gpurun_out/diag_$t.log 2>&1 || { echo "FAIL $t"; tail -3 gpurun_out/diag_$t.log; exit 1; }
  f=$(find gpurun_out/diag_$t -name "*kernel_stats.csv" | head -1)
  echo "== $t"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'rpass' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', round(float(r['TotalDurationNs'])/3e6,2), 'ms/run')
"
done

cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
BRD_LIB=tools/diaglib/wide.so timeout -k 10 240 python3 tools/blk_check.py > gpurun_out/wide_check.log 2>&1 || { echo "FAIL check"; tail -20 gpurun_out/wide_check.log; exit 1; }
tail -15 gpurun_out/wide_check.log
for lib in svdsolver_amd/lib/libbrd_hip.so tools/diaglib/wide.so tools/diaglib/wide6.so; do
  t=$(basename $lib .so)
  BRD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wd_$t -o run -- python3 tools/rp_diag.py > gpurun_out/wd_$t.log 2>&1 || { echo "FAIL $t"; tail -3 gpurun_out/wd_$t.log; exit 1; }
  f=$(find gpurun_out/wd_$t -name "*kernel_stats.csv" | head -1)
  echo "== $t"; python3 -c "
import csv,sys
tot=0
for r in csv.DictReader(open('$f')):
    tot+=float(r['TotalDurationNs'])
    if 'rpass' in r['Name'] or 'blkupd' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', round(float(r['TotalDurationNs'])/3e6,2), 'ms/run')
print('all kernels ms/run', round(tot/3e6,2))
"
done

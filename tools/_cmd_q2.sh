cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_parity.py -k "blocked or structured or extreme or fixture or gen1024" > gpurun_out/q2_tests.log 2>&1 || { echo "FAIL tests"; tail -30 gpurun_out/q2_tests.log; exit 1; }
tail -3 gpurun_out/q2_tests.log
timeout -k 10 240 python3 tools/blk_check.py > gpurun_out/q2_check.log 2>&1 || { echo "FAIL check"; tail -20 gpurun_out/q2_check.log; exit 1; }
tail -10 gpurun_out/q2_check.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q2_prof -o run -- python3 tools/rp_diag.py > gpurun_out/q2_prof.log 2>&1 || { echo "FAIL prof"; tail -3 gpurun_out/q2_prof.log; exit 1; }
f=$(find gpurun_out/q2_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
tot=0
for r in csv.DictReader(open('$f')):
    tot+=float(r['TotalDurationNs'])
    print(r['Name'][:50].ljust(50), r['Calls'].rjust(6), str(round(float(r['AverageNs'])/1e3,1)).rjust(8), 'us', round(float(r['TotalDurationNs'])/3e6,2), 'ms/run')
print('all kernels ms/run', round(tot/3e6,2))
"

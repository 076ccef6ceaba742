# kbench A/B at several sizes (developer tool): bash tools/kbab_n.sh "<binaries>" "<sizes>" [dtype]
cd $GRAFT_REPO_ROOT
for n in $2; do for bin in $1; do
  timeout -k 5 60 tools/$bin $n ${3:-f64} 256 $((n - 32)) > gpurun_out/kbn_${bin}_$n.log 2>&1 || exit 1
  python3 - gpurun_out/kbn_${bin}_$n.log $bin $n <<'PY'
import re, sys
v = {0: [], 1: []}
for line in open(sys.argv[1]):
    m = 'apply' in line and re.search(r'trans=(\d).*?: ([\d.]+) us', line)
    if m: v[int(m.group(1))].append(float(m.group(2)))
print(sys.argv[2], sys.argv[3], 'trans0 %.1f us  trans1 %.1f us' % (sorted(v[0])[1], sorted(v[1])[1]))
PY
done; done

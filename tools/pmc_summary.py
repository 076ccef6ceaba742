"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
KiB per dispatch).  gfx950: FETCH_SIZE counts 64 B per 128-B request of wide
coalesced reads (MI355X_MICROARCH.md, HBM), so 2x FETCH_SIZE is also printed."""
import csv
import glob
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(lambda: [0, 0.0])
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name", counter) != counter:
                continue
            k = r["Kernel_Name"]
            acc[k][0] += 1
            acc[k][1] += float(r["Counter_Value"])
    return acc


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':60s} {'disp':>6s} {'FETCH MiB/disp':>15s} {'2xFETCH':>10s} {'WRITE MiB/disp':>15s}")
for k in sorted(fetch, key=lambda k: -fetch[k][1]):
    n, f = fetch[k]
    w = write.get(k, [1, 0.0])
    print(f"{k[:60]:60s} {n:6d} {f / n / 1024:15.3f} {2 * f / n / 1024:10.3f} {w[1] / max(w[0], 1) / 1024:15.3f}")

"""Average duration (us) per kernel across rocprofv3 kernel traces (developer
tool; pairs with tools/rp_trace_ab.sh): kavg.py FILTER LABEL=DIR ... -> one row
per kernel whose name contains FILTER, one column per trace."""
import csv, glob, sys
from collections import defaultdict

flt = sys.argv[1]
res, names = {}, set()
for a in sys.argv[2:]:
    lab, d = a.split("=", 1)
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt in n:
            k = n.split("(")[0].replace("void ", "")
            acc[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
            acc[k][1] += 1
            names.add(k)
    res[lab] = acc
labs = list(res)
print(f"{'kernel':54s}" + "".join(f"{l:>14s}" for l in labs))
for k in sorted(names):
    print(f"{k[:54]:54s}" + "".join(f"{(res[l][k][0] / res[l][k][1] if res[l][k][1] else 0):14.2f}" for l in labs))

"""Per-panel read-pass durations (us) of one reduction from rocprofv3 kernel
traces (developer tool; tools/rp_trace_ab.sh): LABEL=DIR ... -> a table of Y / X
pass durations at a few panel indices, and the sums."""
import csv, glob, sys

def passes(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_rpass" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    y = [dur(r) for r in rows if "true" in r["Kernel_Name"]]
    x = [dur(r) for r in rows if "false" in r["Kernel_Name"]]
    return y[-252:], x[-252:]

res = {}
for a in sys.argv[1:]:
    lab, d = a.split("=", 1)
    res[lab] = passes(d)
labs = list(res)
print("panel " + " ".join(f"{l + ' Y':>12}{l + ' X':>12}" for l in labs))
for p in [0, 1, 2, 3, 4, 25, 50, 100, 150, 200, 225, 250]:
    print(f"{p:5d} " + " ".join(f"{res[l][0][p]:12.1f}{res[l][1][p]:12.1f}" for l in labs))
print("sum   " + " ".join(f"{sum(res[l][0]) / 1e3:11.2f}m{sum(res[l][1]) / 1e3:11.2f}m" for l in labs))
print("tail150+ " + " ".join(f"{(sum(res[l][0][150:]) + sum(res[l][1][150:])) / 1e3:20.2f}m" for l in labs))

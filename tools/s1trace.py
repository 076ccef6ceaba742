"""Stage-1 per-panel time breakdown from a rocprofv3 kernel trace (developer
tool).  usage: python tools/s1trace.py <kernel_trace.csv> [n=8192] [b=32]
Groups the dispatches of ONE ge2band call (the last one in the trace) by panel
side and reports, per range of panels, factor / apply / gap time."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
b = int(sys.argv[3]) if len(sys.argv) > 3 else 32
rows = list(csv.DictReader(open(path)))
rows = [r for r in rows if "brd::k_" in r["Kernel_Name"] and "band2bd" not in r["Kernel_Name"]
        and "extract" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last ge2band: 2 * n / b panel sides; each side starts with a k_factor launch
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void brd::k_factor")]
sides = 2 * ((n + b - 1) // b) - 1
first = starts[-sides]
seq = rows[first:]
side_idx = -1
acc = defaultdict(lambda: defaultdict(float))
prev_end = None
for r in seq:
    nm = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if nm.startswith("void brd::k_factor"):
        side_idx += 1
    panel = side_idx // 2
    grp = panel * 8 // (n // b)     # 8 ranges of panels
    kind = "factor" if nm.startswith("void brd::k_factor") else ("apply_factor" if "apply_factor" in nm else "apply")
    acc[grp][kind] += (e - s) / 1e3
    if prev_end is not None:
        acc[grp]["gap"] += max(0, s - prev_end) / 1e3
    acc[grp]["launches"] += 1
    prev_end = e
tot = defaultdict(float)
print(f"{'panels':>14s} {'factor':>9s} {'apply_f':>9s} {'apply':>9s} {'gap':>8s} {'launch':>7s}  (us)")
for g in sorted(acc):
    a = acc[g]
    p0, p1 = g * (n // b) // 8, (g + 1) * (n // b) // 8
    print(f"{p0:6d}..{p1:6d} {a['factor']:9.0f} {a['apply_factor']:9.0f} {a['apply']:9.0f} {a['gap']:8.0f} {int(a['launches']):7d}")
    for k, v in a.items():
        tot[k] += v
print(f"{'total':>14s} {tot['factor']:9.0f} {tot['apply_factor']:9.0f} {tot['apply']:9.0f} {tot['gap']:8.0f} {int(tot['launches']):7d}")
print(f"span {(int(seq[-1]['End_Timestamp']) - int(seq[0]['Start_Timestamp'])) / 1e3:.0f} us")

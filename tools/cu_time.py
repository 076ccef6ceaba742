"""CU time per kernel family in a rocprofv3 kernel trace (developer tool).

In a stream of reductions every stage-1 / stage-2 workgroup holds a whole CU
(LDS >= 88 KB), so a launch's CU time is about (workgroups, at most the CUs)
x its duration.  Over the last `frac` of the trace (the timed region) this
prints, per family: launches, summed duration, union busy time, and the CU
time as a share of (window x 256 CUs) -- where the chip's time goes.
usage: python tools/cu_time.py <kernel_trace.csv> [frac=0.5] [cus=256]"""
import csv
import sys

path = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
CUS = int(sys.argv[3]) if len(sys.argv) > 3 else 256


def fam(n):
    for k in ("k_sweeps", "band2bd", "k_rpass", "k_blkupd", "k_prep_qr", "k_prep_lq", "k_cqr_gram", "k_cqr_q1",
              "k_cqr_v", "k_vsum", "k_apply", "k_factor"):
        if k in n:
            return k
    return "other"


rows = []
for r in csv.DictReader(open(path)):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gx = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    wx = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
    wgs = max(1, gx // max(wx, 1))
    rows.append((s, e, r["Kernel_Name"], wgs))
rows.sort()
t0, t1 = rows[0][0], max(e for _, e, _, _ in rows)
lo = t1 - (t1 - t0) * frac
rows = [(max(s, lo), e, n, w) for s, e, n, w in rows if e > lo]
win = t1 - lo


def union(xs):
    tot, cs, ce = 0, None, None
    for s, e in sorted(xs):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


fams = {}
for s, e, n, w in rows:
    fams.setdefault(fam(n), []).append((s, e, w))
print(f"window {win / 1e6:.2f} ms, {len(rows)} launches")
tot_cu = 0.0
for f, xs in sorted(fams.items(), key=lambda kv: -sum((e - s) * min(w, CUS) for s, e, w in kv[1])):
    cu = sum((e - s) * min(w, CUS) for s, e, w in xs)
    tot_cu += cu
    avgw = sum(w for _, _, w in xs) / len(xs)
    print(f"  {f:11s} n {len(xs):6d} sum {sum(e - s for s, e, _ in xs) / 1e6:9.2f} ms  union "
          f"{union([(s, e) for s, e, _ in xs]) / 1e6:8.2f} ms  avg wg {avgw:7.1f}  avg us "
          f"{sum(e - s for s, e, _ in xs) / len(xs) / 1e3:7.1f}  CU share {cu / (win * CUS):6.3f}")
print(f"  total CU share {tot_cu / (win * CUS):.3f} (>1 means workgroups shared CUs or the estimate's tails)")

# timeline: CU occupancy per family in bins (whole trace)
if len(sys.argv) > 4:
    binus = float(sys.argv[4])
    allrows = []
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gx = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        wx = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
        allrows.append((s, e, fam(r["Kernel_Name"]), max(1, gx // max(wx, 1)), r.get("Queue_Id", "?")))
    T0 = min(s for s, _, _, _, _ in allrows)
    T1 = max(e for _, e, _, _, _ in allrows)
    nb = int((T1 - T0) / (binus * 1e3)) + 1
    keys = ["k_sweeps", "k_rpass", "k_blkupd", "k_prep_qr", "k_prep_lq", "k_cqr_q1", "k_cqr_v", "other"]
    occ = [[0.0] * len(keys) for _ in range(nb)]
    qs = [set() for _ in range(nb)]
    for s, e, f, w, qid in allrows:
        k = keys.index(f) if f in keys else len(keys) - 1
        b0, b1 = int((s - T0) / (binus * 1e3)), int((e - T0) / (binus * 1e3))
        for bb in range(b0, b1 + 1):
            lo_ = max(s, T0 + bb * binus * 1e3)
            hi_ = min(e, T0 + (bb + 1) * binus * 1e3)
            if hi_ > lo_:
                occ[bb][k] += (hi_ - lo_) * min(w, CUS) / (binus * 1e3)
                if f != "k_sweeps":
                    qs[bb].add(qid)
    print("bin_ms " + " ".join(f"{k[:9]:>9s}" for k in keys) + "  s1queues")
    for bb in range(nb):
        print(f"{bb * binus / 1e3:6.1f} " + " ".join(f"{v:9.1f}" for v in occ[bb]) + f"  {len(qs[bb])}")

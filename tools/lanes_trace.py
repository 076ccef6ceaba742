"""Concurrency of a pipelined (multi-lane) bench run from a rocprofv3 kernel
trace (developer tool): union busy time per kernel family and overall, over
the last `--span` fraction of the trace (the timed region).
usage: python tools/lanes_trace.py <kernel_trace.csv> [tail_fraction=0.5]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
iv.sort()
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
lo = t1 - (t1 - t0) * frac
iv = [(max(s, lo), e, n) for s, e, n in iv if e > lo]


def fam(n):
    if "band2bd" in n:
        return "stage2"
    for k in ("k_rpass", "k_blkupd", "k_prep", "k_cqr", "k_vsum"):
        if k in n:
            return k
    if "k_apply_factor" in n:
        return "apply_factor"
    if "k_apply" in n:
        return "apply"
    if "k_factor" in n:
        return "factor"
    return "other"


def union(xs):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(xs):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


span = t1 - lo
fams = {}
for s, e, n in iv:
    fams.setdefault(fam(n), []).append((s, e))
print(f"window {span / 1e6:.1f} ms; union busy {union([(s, e) for s, e, _ in iv]) / 1e6:.1f} ms")
for f, xs in sorted(fams.items()):
    print(f"  {f:13s} launches {len(xs):6d} sum {sum(e - s for s, e in xs) / 1e6:9.1f} ms  union {union(xs) / 1e6:8.1f} ms")
s1 = fams.get("apply", []) + fams.get("apply_factor", []) + fams.get("factor", [])
print(f"  stage-1 union {union(s1) / 1e6:.1f} ms; apply-family union "
      f"{union(fams.get('apply', []) + fams.get('apply_factor', [])) / 1e6:.1f} ms")

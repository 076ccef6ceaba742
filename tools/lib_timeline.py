"""CU occupancy of a stream of reductions from the library's own launch
timeline (developer tool; rocprofv3's kernel trace serialises the lanes).
Record it with BRD_PROF_TRACE=<file> around a profiled pass, e.g.
    BRD_PROF_TRACE=gpurun_out/tl.txt python bench.py --one-at-a-time off
(the profiled pass then repeats the stream with per-launch events).
Every stage-1 / stage-2 workgroup holds a whole CU (LDS), so a launch's CU
time is min(workgroups, CUs) x duration; stage 2 (grid unknown here) counts
its reservation.
usage: python tools/lib_timeline.py <file> [bin_ms=20] [cus=256] [s2_cus=32]"""
import sys

path = sys.argv[1]
binms = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
CUS = int(sys.argv[3]) if len(sys.argv) > 3 else 256
S2 = int(sys.argv[4]) if len(sys.argv) > 4 else 32
rows = []
for ln in open(path):
    k, g, a, b = ln.split()[:4]
    g = int(g) or (S2 if k.startswith("s2") else 1)
    rows.append((float(a), float(b), k, min(g, CUS)))
T0 = min(a for a, _, _, _ in rows)
T1 = max(b for _, b, _, _ in rows)
win = T1 - T0
kinds = sorted({k for _, _, k, _ in rows})
print(f"window {win:.1f} ms, {len(rows)} launches")
tot = 0.0
for k in kinds:
    xs = [(a, b, g) for a, b, kk, g in rows if kk == k]
    cu = sum((b - a) * g for a, b, g in xs)
    tot += cu
    print(f"  {k:13s} n {len(xs):6d} sum {sum(b - a for a, b, _ in xs):9.1f} ms  avg us "
          f"{1e3 * sum(b - a for a, b, _ in xs) / len(xs):8.1f}  avg wg {sum(g for *_, g in xs) / len(xs):6.1f}"
          f"  CU share {cu / (win * CUS):.3f}")
print(f"  total CU share {tot / (win * CUS):.3f}")
nb = int(win / binms) + 1
occ = [[0.0] * len(kinds) for _ in range(nb)]
for a, b, k, g in rows:
    ki = kinds.index(k)
    for bb in range(int((a - T0) / binms), int((b - T0) / binms) + 1):
        lo, hi = max(a, T0 + bb * binms), min(b, T0 + (bb + 1) * binms)
        if hi > lo:
            occ[bb][ki] += (hi - lo) * g / binms
print("  t_ms " + " ".join(f"{k[:11]:>11s}" for k in kinds) + "   total")
for bb in range(nb):
    print(f"{bb * binms:6.0f} " + " ".join(f"{v:11.1f}" for v in occ[bb]) + f" {sum(occ[bb]):7.1f}")

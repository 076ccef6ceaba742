"""Stage-2 ring footprint of the reference's window geometry (developer
tool): for each bundle of S consecutive sweeps, the diagonals (column - row)
each row's windows touch (read or write) within that bundle.  The LDS ring
of k_sweeps stores diagonals -31 .. 63 per row (pitch 96 at b = 32); a
narrower pitch would need every row's per-bundle span below it.
Geometry: svd_parallel.h:640-687 (brd_p2), as oracle/brd_oracle_impl.h.
usage: python tools/s2_ring_span.py [n=1024] [b=32] [S=3]"""
import collections
import sys


def windows(n, b, i):
    bs = b + 1
    out = []
    li1, li2, lj1, lj2 = i, min(i + bs, n), i + 1, min(i + bs, n)
    out.append((li1, li2, lj1, lj2))
    lj2 = min(i + bs + bs - 1, n)
    li1 = li1 + 1
    lj1 = i + 1
    out.append((li1, li2, lj1, lj2))
    for _ in range((n - lj2) // (bs - 1) + 1):
        end_i, start_j, end_j3 = min(li2 + bs - 1, n), min(lj1 + bs - 1, n), min(lj2 + bs - 1, n)
        ri1, ri2, rj1, rj2 = li1, end_i, start_j, lj2
        li1, li2, lj1, lj2 = li2, end_i, start_j, end_j3
        if rj2 > rj1:
            out.append((ri1, ri2, rj1, rj2))
        if lj2 > lj1:
            out.append((li1, li2, lj1, lj2))
    return out


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
b = int(sys.argv[2]) if len(sys.argv) > 2 else 32
S = int(sys.argv[3]) if len(sys.argv) > 3 else 3
spans = collections.Counter()
for beta in range((n - 1 + S - 1) // S):
    lo, hi = {}, {}
    for i in range(beta * S, min(beta * S + S, n - 1)):
        for i1, i2, j1, j2 in windows(n, b, i):
            for r in range(i1, i2):
                lo[r] = min(lo.get(r, 1 << 30), j1 - r)
                hi[r] = max(hi.get(r, -(1 << 30)), j2 - 1 - r)
    for r in lo:
        if 3 * b < r < n - 3 * b:   # interior rows
            spans[(lo[r], hi[r])] += 1
tot = sum(spans.values())
print(f"n={n} b={b} S={S}: {tot} (bundle, interior row) pairs")
for (a, z), c in spans.most_common(6):
    print(f"  diagonals {a:4d} .. {z:3d} (span {z - a + 1:3d}): {c} ({100.0 * c / tot:.1f} %)")
print(f"  widest span {max(z - a + 1 for a, z in spans)}")

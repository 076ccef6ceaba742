"""Read-pass launches of a one-at-a-time run from the library's launch
timeline (BRD_PROF_TRACE, bench.py --pipeline off): duration against the
algorithmic bytes, a least-squares t = t0 + bytes / BW fit over the passes
(the fixed cost per pass and the streaming rate), and the time split by
pass size.  usage: python tools/rpass_fit.py <trace> [kind=s1_rpass]"""
import sys

import numpy as np

kind = sys.argv[2] if len(sys.argv) > 2 else "s1_rpass"
rows = [ln.split() for ln in open(sys.argv[1])]
xs = np.array([(float(r[4]), float(r[3]) - float(r[2])) for r in rows if r[0] == kind and len(r) > 4])
by, ms = xs[:, 0], xs[:, 1]
A = np.stack([np.ones_like(by), by], axis=1)
(t0, inv), *_ = np.linalg.lstsq(A, ms, rcond=None)
print(f"{kind}: {len(ms)} launches, {ms.sum():.2f} ms, {by.sum() / 1e9:.2f} GB -> {by.sum() / ms.sum() / 1e9:.0f} GB/s")
print(f"fit t = {t0 * 1e3:.1f} us + bytes / {1 / inv / 1e9:.0f} GB/s")
for lo, hi in [(0, 16e6), (16e6, 64e6), (64e6, 256e6), (256e6, 1e12)]:
    m = (by >= lo) & (by < hi)
    if m.any():
        print(f"  {lo / 1e6:5.0f}-{hi / 1e6:5.0f} MB: {m.sum():4d} passes {ms[m].sum():7.2f} ms "
              f"{by[m].sum() / ms[m].sum() / 1e9:6.0f} GB/s  avg {1e3 * ms[m].mean():6.1f} us")

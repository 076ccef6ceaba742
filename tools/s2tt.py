"""Stage-2 per-task timeline of two consecutive bundles (developer tool).

Reads gpurun_out/s2tt.bin written by tools/s2bench (BRD_STAMPS build): per
compute wave and task the s_memrealtime stamps [start, rows-ready, done] of
bundles kTB0 and kTB0+1, and the publication logs (loader `loaded`, writer
`rows_done`, poller `avail`).  Prints, for a range of the lead's tasks of the
second bundle, where its time went and which hand-off it waited on.

usage: python tools/s2tt.py [gpurun_out/s2tt.bin] [t0] [t1]
"""
import sys

import numpy as np

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/s2tt.bin"
t0 = int(sys.argv[2]) if len(sys.argv) > 2 else 100
t1 = int(sys.argv[3]) if len(sys.argv) > 3 else 130
raw = open(path, "rb").read()
ntt = 2 * 4 * 520 * 3
tt = np.frombuffer(raw, np.uint64, ntt).reshape(2, 4, 520, 3).astype(np.int64)
pub = np.frombuffer(raw, np.uint64, 2 * 3 * 2048 * 2, ntt * 8).reshape(2, 3, 2048, 2).astype(np.int64)
npub = np.frombuffer(raw, np.int32, 6, (ntt + 2 * 3 * 2048 * 2) * 8).reshape(2, 3)
base = tt[0, 0, 0, 0]
us = lambda x: (x - base) / 100.0
names = ["loaded", "rows_done", "avail"]


def at(bd, kind, time):
    """value of log (bd, kind) at time (last publication <= time), and when it was published"""
    m = min(int(npub[bd, kind]), 2048)
    ts, vs = pub[bd, kind, :m, 0], pub[bd, kind, :m, 1]
    k = np.searchsorted(ts, time, side="right") - 1
    return (int(vs[k]), us(ts[k])) if k >= 0 else (-1, -1.0)


nw = int((tt[1, :, 0, 0] > 0).sum())
print(f"compute waves with stamps: {nw}; log sizes {npub.tolist()}")
for w in range(nw):
    d = tt[1, w]
    ok = d[:, 2] > 0
    nt = int(ok.sum())
    work = (d[:nt, 2] - d[:nt, 1]).mean() / 100.0
    wprev = (d[:nt, 1] - d[:nt, 0]).mean() / 100.0
    print(f"bundle+1 wave {w}: {nt} tasks, mean work {work:.3f} us, mean wait {wprev:.3f} us, "
          f"span {(d[nt - 1, 2] - d[0, 0]) / 100.0:.1f} us")
print(f"\nlead of bundle+1, tasks {t0}..{t1}: start  wait(rows)  work | loaded(+pub time) avail  "
      f"rows_done(b)  rows_done(b+1) | trail(b) task")
for t in range(t0, t1):
    s, r, e = tt[1, 0, t]
    ld, ldt = at(1, 0, r)
    av, avt = at(1, 2, r)
    rd0, rd0t = at(0, 1, r)
    rd1, rd1t = at(1, 1, r)
    trail = int(np.searchsorted(tt[0, nw - 1, :, 2], r, side="right"))
    print(f"  t={t:3d} {us(s):9.2f} {(r - s) / 100:7.2f} {(e - r) / 100:6.2f} | "
          f"{ld:6d} ({ldt:9.2f}) {av:6d} ({avt:9.2f}) {rd0:6d} ({rd0t:9.2f}) {rd1:6d} | {trail}")

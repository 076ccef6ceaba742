"""Stage-2 in-bundle lag analysis (developer tool): from gpurun_out/s2tt.bin
(tools/s2bench, STAMPS build) print, for tasks t0..t1 of bundle kTB0+1, each
compute wave's [start, ready, end] (us) and, for the follower sweep, how long
after the lead's task t+3 ended the follower's task t became ready.
usage: python tools/s2lag.py W [t0] [t1]"""
import sys

import numpy as np

W = int(sys.argv[1])
t0 = int(sys.argv[2]) if len(sys.argv) > 2 else 100
t1 = int(sys.argv[3]) if len(sys.argv) > 3 else 112
raw = open("gpurun_out/s2tt.bin", "rb").read()
tt = np.frombuffer(raw, np.uint64, 2 * 4 * 520 * 3).reshape(2, 4, 520, 3).astype(np.int64)
base = tt[1, 0, 0, 0]
us = lambda x: (x - base) / 100.0
nw = int((tt[1, :, 0, 0] > 0).sum())
print(f"waves with stamps: {nw} (W={W})")
for t in range(t0, t1):
    row = []
    for w in range(nw):
        s, r, e = tt[1, w, t]
        row.append(f"w{w} {us(s):8.2f} {us(r):8.2f} {us(e):8.2f}")
    extra = ""
    if nw >= 2 * W:
        lead_end = max(tt[1, w, t + 3, 2] for w in range(W))
        fol_ready = min(tt[1, w, t, 1] for w in range(W, 2 * W))
        fol_start = min(tt[1, w, t, 0] for w in range(W, 2 * W))
        extra = f" | follower ready - lead(t+3) end {(fol_ready - lead_end) / 100:6.2f}  start->ready {(fol_ready - fol_start) / 100:6.2f}"
    print(f"t={t:3d} " + " | ".join(row) + extra)
# mean per-task durations (start of t+1 - start of t) per wave
for w in range(nw):
    st = tt[1, w, :, 0]
    ok = st > 0
    k = int(ok.sum())
    d = np.diff(st[:k]) / 100.0
    wk = (tt[1, w, :k, 2] - tt[1, w, :k, 1]) / 100.0
    print(f"wave {w}: {k} tasks, mean start-to-start {d.mean():.3f} us, mean work {wk.mean():.3f} us")

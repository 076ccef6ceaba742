"""Stage-2 k_sweeps timeline (developer tool; needs a BRD_S2TRACE build):
    bash tools/variant_lib.sh s2tr -DBRD_S2TRACE
    BRD_LIB=tools/ablib/s2tr.so python tools/s2trace.py [N] [f32]
Runs one band2bd at N, reads the per-task / per-publication stamps of bundles
600..603 (chip-wide 100 MHz clock) and prints where each sweep's time goes
(lag wait, row wait, window work) and the hand-off chain of rows between
consecutive bundles: upstream trail releases row X -> upstream writer's
rows_done > X -> downstream poller sees it -> downstream loader has it in the
ring -> downstream lead starts the first window that needs it."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402
from svdsolver_amd import brd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dt = torch.float32 if (len(sys.argv) > 2 and sys.argv[2] == "f32") else torch.float64
B0, NB, NT, NP = 600, 4, 600, 1024
b = 32


def windows_of(i, m, n, bb=32):
    bs = bb + 1
    tl = (i, min(i + bs, m), i + 1, min(i + bs, n))
    tasks = [tl]
    tl = (i + 1, min(i + bs, m), i + 1, min(i + 2 * bs - 1, n))
    tasks.append(tl)
    nbtx = (n - tl[3]) // (bs - 1)
    for _ in range(nbtx + 1):
        end_i = min(tl[1] + bs - 1, m)
        sj = min(tl[2] + bs - 1, n)
        ej3 = min(tl[3] + bs - 1, n)
        tasks += [(tl[0], end_i, sj, tl[3]), (tl[1], end_i, sj, ej3)]
        tl = (tl[1], end_i, sj, ej3)
    return tasks


def next_top(tasks, t, m):
    if t + 1 >= len(tasks):
        return m
    return tasks[t + 1][0]


L = ctypes.CDLL(brd.LIB_PATH)
fn = L.brd_dbg_s2trace
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
fn.restype = ctypes.c_int
sz_task = NB * 12 * NT * 4 * 8
sz_pub = NB * 8 * NP * 2 * 8
sz_npub = NB * 8 * 4
sz = sz_task + sz_pub + sz_npub + 4 + NB * 4 * 8   # (padding before the 8-byte array)
buf = (ctypes.c_ubyte * (sz + 64 + NB * 256 * 8 * 8))()

g = torch.Generator(device="cuda").manual_seed(n)
A = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
S.ge2band(A, b)
for rep in range(2):
    W = A.clone()
    assert fn(None, 0, 1) == 0
    torch.cuda.synchronize()
    d, e = S.band2bd(W, b)
    torch.cuda.synchronize()
assert fn(buf, sz + 64 + NB * 256 * 8 * 8, 0) == 0
raw = bytes(buf)
task = np.frombuffer(raw, dtype=np.uint64, count=NB * 12 * NT * 4).reshape(NB, 12, NT, 4).astype(np.int64)
off = sz_task
pub = np.frombuffer(raw, dtype=np.uint64, count=NB * 8 * NP * 2, offset=off).reshape(NB, 8, NP, 2).astype(np.int64)
off += sz_pub
npub = np.frombuffer(raw, dtype=np.int32, count=NB * 8, offset=off).reshape(NB, 8)
off += sz_npub
off = (off + 7) // 8 * 8
bund = np.frombuffer(raw, dtype=np.uint64, count=NB * 4, offset=off).reshape(NB, 4).astype(np.int64)
wrs = np.frombuffer(raw, dtype=np.uint64, count=NB * 256 * 8, offset=off + NB * 4 * 8).reshape(NB, 256, 8).astype(np.int64)

S_ = None
for k in range(12):
    if task[0, k, 0, 0] == 0:
        S_ = k
        break
S_ = S_ or 12
print(f"n={n} {dt}: sweeps per bundle {S_}; bundles {B0}..{B0 + NB - 1}: "
      f"blocks {list(bund[:, 2])} xcc {list(bund[:, 3])}; bundle time "
      f"{[round((bund[k, 1] - bund[k, 0]) / 100.0, 1) for k in range(NB)]} us; starts "
      f"{[round((bund[k, 0] - bund[0, 0]) / 100.0, 1) for k in range(NB)]} us")
us = 0.01   # 100 MHz ticks -> us
for k in range(NB):
    beta = B0 + k
    parts = []
    for w in range(S_):
        i = beta * S_ + w
        tasks = windows_of(i, n, n)
        nt = min(len(tasks), NT)
        T = task[k, w, :nt]
        live = [t for t in range(2, nt - 4) if tasks[t][1] > tasks[t][0] and tasks[t][3] > tasks[t][2]]
        lag = np.array([T[t, 1] - T[t, 0] for t in live]) * us
        rows = np.array([T[t, 2] - T[t, 1] for t in live]) * us
        work = np.array([T[t, 3] - T[t, 2] for t in live]) * us
        step = np.array([T[t + 1, 0] - T[t, 0] for t in live]) * us
        wr = np.array([T[t, 3] - T[t, 2] for t in live if t % 2 == 0]) * us
        wl = np.array([T[t, 3] - T[t, 2] for t in live if t % 2 == 1]) * us
        parts.append(f"  sweep {w}: step {step.mean():.2f} = lag {lag.mean():.2f} + rows {rows.mean():.2f} + work "
                     f"{work.mean():.2f} (right {wr.mean():.2f} left {wl.mean():.2f}) us/task, sweep "
                     f"{(T[nt - 1, 3] - T[0, 0]) * us:.0f} us")
    print(f"bundle {beta}:")
    print("\n".join(parts))
    print(f"  pubs: loader {npub[k, 0]} writer {npub[k, 1]} poller {npub[k, 2]}")

# hand-off chain from bundle B0+k (upstream) to B0+k+1 (downstream)
for k in range(NB - 1):
    up, dn = B0 + k, B0 + k + 1
    trail = up * S_ + S_ - 1
    lead = dn * S_
    ttasks = windows_of(trail, n, n)
    ltasks = windows_of(lead, n, n)
    Tt = task[k, S_ - 1]
    Tl = task[k + 1, 0]

    def first_pub(kk, kind, X):
        m = npub[kk, kind]
        v = pub[kk, kind, :m]
        idx = np.nonzero(v[:, 1] > X)[0]
        return v[idx[0], 0] if len(idx) else None

    rows = []
    for X in range(lead + 600, min(n - 200, lead + 5000), 97):
        # trail releases X when its front (next window's top row) passes X
        rel = None
        for t in range(min(len(ttasks), NT)):
            if next_top(ttasks, t, n) > X:
                rel = Tt[t, 3]
                break
        use = None
        for t in range(min(len(ltasks), NT)):
            if ltasks[t][1] > X:
                use = (Tl[t, 1], Tl[t, 2])
                break
        wrt = first_pub(k, 1, X)
        pol = first_pub(k + 1, 2, X)
        lod = first_pub(k + 1, 0, X)
        if None in (rel, use, wrt, pol, lod):
            continue
        rows.append((wrt - rel, pol - wrt, lod - pol, use[1] - lod, use[1] - use[0], use[1] - rel))
    if rows:
        a = np.array(rows, dtype=np.float64) * us
        med = np.median(a, axis=0)
        print(f"hop {up}->{dn} (median over {len(a)} rows, us): released->rows_done {med[0]:.2f}, ->poller {med[1]:.2f}, "
              f"->loaded {med[2]:.2f}, ->lead ready {med[3]:.2f} (lead waited on rows {med[4]:.2f}); total {med[5]:.2f}")

# raw view: bundle B0+1, every compute wave: start of selected tasks relative to the bundle start
k = 1
t0b = bund[k, 0]
for w in range(S_):
    i = (B0 + k) * S_ + w
    tasks = windows_of(i, n, n)
    nt = min(len(tasks), NT)
    T = task[k, w, :nt]
    sel = [0, 1, 2, 3, 4, 10, 50, 100, 200, 300] + list(range(max(0, nt - 8), nt))
    sel = sorted(set(t for t in sel if t < nt))
    print(f"bundle {B0 + k} sweep {w} ({nt} tasks): " + ", ".join(
        f"t{t}:{(T[t, 0] - t0b) * us:.0f}/{(T[t, 2] - t0b) * us:.0f}/{(T[t, 3] - t0b) * us:.0f}" for t in sel))
for kind, nm in ((0, "loaded"), (1, "rows_done"), (2, "avail"), (3, "claim"), (4, "issued"), (5, "ldissue"), (6, "freed")):
    m = npub[k, kind]
    v = pub[k, kind, :m]
    idx = sorted(set([0, 1, 2, m // 4, m // 2, 3 * m // 4] + list(range(max(0, m - 6), m))))
    print(f"  {nm}: " + ", ".join(f"{(v[q, 0] - t0b) * us:.0f}us:{v[q, 1]}" for q in idx if q < m))

# per-batch writer timeline (bundle B0+1): claim -> stores issued -> drained (rows_done)
k = 1
def series(kind):
    m = npub[k, kind]
    return pub[k, kind, :m]
cl, iss, dn, fr = series(3), series(4), series(1), series(6)
m = min(len(cl), len(iss), len(dn))
d1 = (iss[:m, 0] - cl[:m, 0]) * us
d2 = (dn[:m, 0] - iss[:m, 0]) * us
print(f"writer per batch (median): claim->issued {np.median(d1):.2f} us, issued->drained+published {np.median(d2):.2f} us; "
      f"batch rows median {np.median(np.diff(np.concatenate([[cl[0, 1]], iss[:m, 1]]))):.0f}")
# loader: issue -> loaded for the same row count
li, lo, av = series(5), series(0), series(2)
lat = []
for q in range(len(li)):
    X = li[q, 1]
    idx = np.nonzero(lo[:, 1] >= X)[0]
    if len(idx):
        lat.append((lo[idx[0], 0] - li[q, 0]) * us)
print(f"loader: issue -> loaded (median over {len(lat)} issues) {np.median(lat):.2f} us; issues per bundle {len(li)}")
# what limited each loader issue: avail or freed + R

W_ = wrs[1]
ok = [q for q in range(256) if W_[q, 0] and W_[q, 7] and W_[q, 6]]
if ok:
    d = np.array([[W_[q, j + 1] - W_[q, j] for j in range(7)] for q in ok]) * us
    print("writer batch phases (median us): claim->rd0 %.2f, ->free0 %.2f, ->st0 %.2f, ->rd1 %.2f, ->free1 %.2f, ->st1 %.2f, ->drained %.2f"
          % tuple(np.median(d, axis=0)))

lim = series(7)
if len(lim):
    v = lim[:, 1]
    print(f"loader issue limited by: avail {np.mean(v % 2 == 0):.2f}, ring {np.mean(v % 2 == 1):.2f}, in-flight cap {np.mean(v >= 2):.2f}")

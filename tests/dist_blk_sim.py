"""TEST INFRASTRUCTURE: numpy restatement of the BLOCKED distributed stage 1
(svdsolver_amd/csrc/brd_stage1_blk.hip, blk_ge2band_dist) -- which rank
computes what and which collectives move it -- so that the sharded data flow
can be checked on CPU with gloo ranks (tests/test_dist.py).  Never imported by
the product path.  The panel QRs are tests/s1_model.py's cholqr_house (the
GPU kernels' CholeskyQR + basis-kernel reconstruction), the per-panel tail
is tests/dist_sim.py.

Layout: global column panel p on rank p mod P (brd_dist.hip).  Lw = [V | X]
(m rows) replicated; Y, U (RwT^T) hold this rank's columns only.  Per panel
j (global panel p, column c):
  1. the owner of p corrects its column panel, CholeskyQR -> V_j, T_j, R;
     BROADCAST of V_j, T_j;
  2. Y pass on this rank's trailing columns (local);
  3. this rank's columns of the corrected row panel, factored by a sharded
     CholeskyQR2 (cholqr_dist): per pass a local 32 x 32 Gram, ALL-GATHER of
     the per-rank Grams summed in rank order (every rank: the same R), local
     Q = P R^-1; the rank holding the band block's columns (panel p+1, rank
     (p+1) mod P: the top block of the panel) finishes the basis-kernel
     reconstruction and BROADCASTS S_j;
  4. X pass partial over this rank's columns (with its part of the Y^T U,
     U^T U corrections); ALL-REDUCE;
block end: the rank-2 nb b update of this rank's trailing columns (local).
"""
import numpy as np

from dist_sim import ge2band_dist_sim, panels_before
from s1_model import blocked_columns, cholqr_house


def cholqr_dist(Ploc, top, root, P, dist, group=None, iters=2):
    """The row panel's QR with its rows sharded over the ranks (this rank's
    rows Ploc; `top`: this rank holds the panel's first k rows): CholeskyQR2
    with all-gathered per-rank Grams, then the basis-kernel form of the
    Householder reconstruction (Ballard et al. 2015; the GPU kernels'
    k_cqr_v): V = Q - [S; 0], T = -S (U^-1 L^-1)^T with Q_t - S = L U, the
    band block S R.  Returns this rank's rows of V, T (broadcast from the
    top rank) and, on the top rank, S R."""
    import torch
    nc, k = Ploc.shape
    mx = torch.tensor([float(np.max(np.abs(Ploc))) if Ploc.size else 0.0], dtype=torch.float64)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    scale = float(mx[0])
    if scale == 0.0:
        V = np.zeros((nc, k))
        if top:
            V[:k, :k] = np.eye(k)
        return V, np.zeros((k, k)), np.zeros((k, k))
    e = np.floor(np.log2(scale))
    Q = Ploc * 2.0 ** (-e)
    R = np.eye(k)
    for _ in range(iters):
        parts = [torch.zeros((k, k), dtype=torch.float64) for _ in range(P)]
        dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(Q.T @ Q)), group=group)
        G = parts[0].numpy().copy()
        for r in range(1, P):
            G = G + parts[r].numpy()
        C = np.linalg.cholesky(G).T          # upper, G = C^T C: the same on every rank
        Q = np.linalg.solve(C.T, Q.T).T
        R = C @ R
    R = R * 2.0 ** e
    tb = np.zeros((k, k))
    Rh = np.zeros((k, k))
    V = Q.copy()
    if top:   # the modified LU of the top block: s_j = -sign(pivot)
        lu = Q[:k].copy()
        S = np.zeros(k)
        for j in range(k):
            s = -1.0 if lu[j, j] >= 0 else 1.0
            S[j] = s
            lu[j, j] -= s
            lu[j + 1:, j] /= lu[j, j]
            lu[j + 1:, j + 1:] -= np.outer(lu[j + 1:, j], lu[j, j + 1:])
        L1 = np.tril(lu, -1) + np.eye(k)
        U = np.triu(lu)
        tb = -np.diag(S) @ np.linalg.inv(L1 @ U).T
        V[:k] -= np.diag(S)
        Rh = np.triu(np.diag(S) @ R)
    t = torch.from_numpy(tb)
    dist.broadcast(t, src=root, group=group)
    return V, t.numpy(), Rh


def global_columns(n, b, P, rank):
    cols = [np.arange(p * b, min(n, p * b + b)) for p in range(rank, (n + b - 1) // b, P)]
    return np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)


def ge2band_blk_dist_sim(A_loc, n, b, rank, P, dist, group=None, nb=4):
    """Blocked distributed dense -> band on this rank's shard (in place),
    then the per-panel distributed tail."""
    import torch
    m, n_loc = A_loc.shape
    gcol = global_columns(n, b, P, rank)
    kend = blocked_columns(n, b, nb)
    k0 = 0
    while k0 < kend:
        V = np.zeros((m, 0)); X = np.zeros((m, 0))
        Y = np.zeros((n_loc, 0)); U = np.zeros((n_loc, 0))
        c = k0
        for _ in range(nb):
            p = c // b
            o, o2 = p % P, (p + 1) % P
            tr = gcol >= c + b                     # this rank's trailing columns
            nc = int(tr.sum())
            # 1. the owner's column panel QR, broadcast of V_j and T_j
            buf = np.zeros((m - c + b, b))
            if rank == o:
                lc = panels_before(p, P, rank) * b
                Pn = A_loc[c:, lc:lc + b] - V[c:] @ Y[lc:lc + b].T - X[c:] @ U[lc:lc + b].T
                Vj, Tj, Rj = cholqr_house(Pn)
                A_loc[c:, lc:lc + b] = 0.0
                A_loc[c:c + b, lc:lc + b] = Rj
                buf[:m - c] = Vj
                buf[m - c:] = Tj
            tb = torch.from_numpy(buf)
            dist.broadcast(tb, src=o, group=group)
            Vj, Tj = tb.numpy()[:m - c], tb.numpy()[m - c:]
            Vf = np.zeros((m, b)); Vf[c:] = Vj
            # 2. Y pass, local
            Yf = np.zeros((n_loc, b))
            Yf[tr] = (A_loc[c:, tr].T @ Vj - Y[tr] @ (V[c:].T @ Vj) - U[tr] @ (X[c:].T @ Vj)) @ Tj
            V = np.hstack([V, Vf]); Y = np.hstack([Y, Yf])
            # 3. the row panel: local columns, a sharded CholeskyQR
            Q = A_loc[c:c + b, tr] - V[c:c + b] @ Y[tr].T - X[c:c + b] @ U[tr].T
            Uj, Sj, Lt = cholqr_dist(Q.T, rank == o2, o2, P, dist, group)
            A_loc[c:c + b, tr] = 0.0
            if rank == o2:
                lc2 = panels_before(p + 1, P, rank) * b
                A_loc[c:c + b, lc2:lc2 + b] = Lt.T
            Uf = np.zeros((n_loc, b)); Uf[tr] = Uj
            # 4. X pass partial over this rank's columns, all-reduced
            Zp = A_loc[c + b:, tr] @ Uj - V[c + b:] @ (Y[tr].T @ Uj) - X[c + b:] @ (U[tr].T @ Uj)
            Zt = torch.from_numpy(np.ascontiguousarray(Zp))
            dist.all_reduce(Zt, group=group)
            Xf = np.zeros((m, b)); Xf[c + b:] = Zt.numpy() @ Sj
            X = np.hstack([X, Xf]); U = np.hstack([U, Uf])
            c += b
        tr = gcol >= c
        A_loc[c:, tr] -= V[c:] @ Y[tr].T + X[c:] @ U[tr].T
        k0 = c
    return ge2band_dist_sim(A_loc, n, b, rank, P, dist, group=group, k_start=kend // b)

"""Test infrastructure: numpy restatement of the distributed stage 1 of
svdsolver_amd/csrc/brd_dist.hip (same panel steps, same collectives through
torch.distributed), so that the algorithm and its communication pattern can
be checked on CPU with gloo.  Never imported by the product path.

Per panel k (owner k mod P), as in brd_dist.hip:
  1. broadcast of the column panel, Householder QR on every rank, owner keeps R;
  2. left update Q^T of each rank's trailing columns;
  3. LQ of the row panel: local Householder QR of the rank's columns
     (transposed), all-gather of the b x b R factors, stack starting with the
     owner of panel k+1, QR of the stack (the root);
  4. right update: local reflectors on the rank's columns, then the root:
     W = sum over ranks of V_root_block^T X_root_block (all-reduce), update.
"""
import numpy as np


def hqr(X):
    """Householder QR, LAPACK conventions (tau = 0 for a zero sub-column):
    X = (I - V T V^T) [R; 0].  Returns V (M x kk), T (kk x kk), R (kk x k)."""
    X = np.array(X, dtype=np.float64, copy=True)
    M, k = X.shape
    kk = min(M, k)
    V = np.zeros((M, kk))
    tau = np.zeros(kk)
    for j in range(kk):
        x = X[j:, j]
        sub2 = float(x[1:] @ x[1:])
        v = np.zeros(M - j)
        v[0] = 1.0
        if sub2 != 0.0:
            nrm = np.sqrt(x[0] * x[0] + sub2)
            alpha = -nrm if x[0] >= 0 else nrm
            u1 = x[0] - alpha
            v[1:] = x[1:] / u1
            tau[j] = -u1 / alpha
            X[j:, j:] -= tau[j] * np.outer(v, v @ X[j:, j:])
        V[j:, j] = v
    T = np.zeros((kk, kk))
    for j in range(kk):
        T[:j, j] = -tau[j] * (T[:j, :j] @ (V[:, :j].T @ V[:, j]))
        T[j, j] = tau[j]
    return V, T, np.triu(X[:kk, :])


class LocalComm:
    """torch.distributed stand-in for a single rank (P = 1)."""

    @staticmethod
    def broadcast(t, src=0, group=None):
        return None

    @staticmethod
    def all_gather(parts, t, group=None):
        parts[0].copy_(t)

    @staticmethod
    def all_reduce(t, group=None):
        return None


def panels_before(g, P, r):
    return (g - r + P - 1) // P if g > r else 0


def ge2band_dist_sim(A_loc, n, b, rank, P, dist, group=None, k_start=0):
    """Distributed dense -> band on this rank's shard (numpy, in place), from
    global panel k_start on."""
    import torch
    m = A_loc.shape[0]
    n_loc = A_loc.shape[1]
    np_ = (n + b - 1) // b
    for k in range(k_start, np_):
        kb = k * b
        bk = min(b, n - kb)
        mp, n2 = m - kb, n - kb - bk
        owner = k % P
        lck = (k // P) * b
        lcs = panels_before(k + 1, P, rank) * b
        nc = n_loc - lcs
        # 1. broadcast + QR of the column panel
        pan = torch.from_numpy(np.ascontiguousarray(A_loc[kb:, lck:lck + bk]) if rank == owner
                               else np.zeros((mp, bk)))
        dist.broadcast(pan, src=owner, group=group)
        V, T, R = hqr(pan.numpy())
        if rank == owner:
            A_loc[kb:, lck:lck + bk] = 0.0
            A_loc[kb:kb + R.shape[0], lck:lck + bk] = R
        if n2 <= 0:
            continue
        # 2. left update
        if nc > 0:
            X = A_loc[kb:, lcs:]
            X -= V @ (T.T @ (V.T @ X))
        # 3. LQ: local QR of the transposed row panel, gathered R, root
        nrow = max(0, min(nc, bk))
        Rpad = np.zeros((bk, bk))
        if nc > 0:
            Vl, Tl, Rl = hqr(A_loc[kb:kb + bk, lcs:].T)
            A_loc[kb:kb + bk, lcs:] = 0.0
            Rpad[:nrow] = Rl[:nrow]
        parts = [torch.zeros((bk, bk), dtype=torch.float64) for _ in range(P)]
        dist.all_gather(parts, torch.from_numpy(Rpad), group=group)
        first = (k + 1) % P
        stack = np.concatenate([parts[(first + s) % P].numpy() for s in range(P)])
        Vr, Tr, Rr = hqr(stack)
        stack_out = np.zeros_like(stack)
        stack_out[:Rr.shape[0]] = Rr
        mypos = (rank - first) % P
        if nrow > 0:
            A_loc[kb:kb + bk, lcs:lcs + nrow] = stack_out[mypos * bk:mypos * bk + nrow].T
        # 4. right update of rows kb+bk..
        m2 = m - kb - bk
        if m2 <= 0:
            continue
        if nc > 0:
            Z = A_loc[kb + bk:, lcs:]
            Z -= ((Z @ Vl) @ Tl) @ Vl.T
        Vb = Vr[mypos * bk:mypos * bk + bk]
        Wp = np.zeros((Vr.shape[1], m2))
        if nrow > 0:
            Wp = Vb[:nrow].T @ A_loc[kb + bk:, lcs:lcs + nrow].T
        Wt = torch.from_numpy(np.ascontiguousarray(Wp))
        dist.all_reduce(Wt, group=group)
        if nrow > 0:
            Xr = A_loc[kb + bk:, lcs:lcs + nrow].T - Vb[:nrow] @ (Tr.T @ Wt.numpy())
            A_loc[kb + bk:, lcs:lcs + nrow] = Xr.T
    return A_loc

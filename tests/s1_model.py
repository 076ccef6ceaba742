"""TEST INFRASTRUCTURE: numpy model of the delayed (two-sided, blocked)
stage-1 reduction that brd_stage1_blk.hip implements on the GPU.

Not the product path -- it is the executable specification the GPU kernels
are checked against step by step, and it is itself checked against the
oracle's band (tests/test_s1_model.py).  See DESIGN.md "Stage 1, blocked".

Dense m x n -> upper band (b super-diagonals).  Panels of b columns are
grouped in blocks of nb panels.  Inside a block the trailing matrix is never
written; it is kept implicitly as

    A_cur = A - V Y^T - X U^T

(V, X: m x (j b), Y, U: n x (j b)) and updated once at block end with one
rank-2 nb b product.  Per panel j (column offset c):

  1. column panel  P = A[c:, c:c+b] - V Y[c:c+b]^T - X U[c:c+b]^T
  2. P = (I - V_j T_j V_j^T) [R; 0]          (cholqr_house: CholeskyQR2 +
                                               Householder reconstruction)
  3. Y_j = (A^T V_j - Y (V^T V_j) - U (X^T V_j)) T_j      (a read pass of A)
  4. row panel     Q = A[c:c+b, c+b:] - V[c:c+b] Y^T - X[c:c+b] U^T
  5. Q^T = (I - U_j S_j U_j^T) [L^T; 0]
  6. X_j = (A U_j - V (Y^T U_j) - X (U^T U_j)) S_j        (a read pass of A)

The reference reduces each panel with per-column Householder kernels and
applies Q / P to the whole trailing matrix every panel
(svd_cuda_2.cu:1117-1220, qr_apply_cuda :1039, lq_apply_cuda :1081); the
band is the same up to the signs of its rows / columns.
"""
from __future__ import annotations

import numpy as np


def cholqr_house(P: np.ndarray, iters: int = 2):
    """QR of a tall m x k panel (m >= k) as a Householder block reflector.

    Returns V (m x k, unit lower trapezoidal), T (k x k upper) and R (k x k
    upper) with (I - V T V^T)^T P = [R; 0].  CholeskyQR2 gives Q with
    orthonormal columns; the modified LU of Q - [S; 0] (Ballard et al.,
    "Reconstructing Householder vectors from TSQR", 2015) gives V = L and
    T = -U S L1^-T, R_house = S R."""
    m, k = P.shape
    dt = P.dtype
    P = P.astype(np.float64)
    scale = np.max(np.abs(P)) if P.size else 0.0
    if scale == 0.0:
        V = np.zeros((m, k)); V[:k, :k] = np.eye(k)
        return V.astype(dt), np.zeros((k, k), dt), np.zeros((k, k), dt)
    e = np.floor(np.log2(scale))
    Ps = P * 2.0 ** (-e)
    Q = Ps
    R = np.eye(k)
    for _ in range(iters):
        G = Q.T @ Q
        C = np.linalg.cholesky(G).T          # upper, G = C^T C
        Q = np.linalg.solve(C.T, Q.T).T      # Q C^-1
        R = C @ R
    R = R * 2.0 ** e
    # modified LU of the top block: s_j = -sign(pivot)
    top = Q[:k].copy()
    S = np.zeros(k)
    for j in range(k):
        s = -1.0 if top[j, j] >= 0 else 1.0
        S[j] = s
        top[j, j] -= s
        top[j + 1:, j] /= top[j, j]
        top[j + 1:, j + 1:] -= np.outer(top[j + 1:, j], top[j, j + 1:])
    L1 = np.tril(top, -1) + np.eye(k)
    U = np.triu(top)
    L2 = np.linalg.solve(U.T, Q[k:].T).T     # Q2 U^-1
    V = np.vstack([L1, L2])
    T = -U @ np.diag(S) @ np.linalg.inv(L1.T)
    Rh = np.diag(S) @ R
    return V.astype(dt), np.triu(T).astype(dt), np.triu(Rh).astype(dt)


def _tail_unblocked(A: np.ndarray, k0: int, b: int) -> None:
    """Panels from column k0 on, one at a time (Householder QR / LQ of each
    panel applied to the whole trailing matrix: the reference's structure).
    The GPU runs these last panels with the per-panel tree kernels."""
    m, n = A.shape
    c = k0
    while c < n:
        bk = min(b, n - c)
        Qf, R = np.linalg.qr(A[c:, c:c + bk].astype(np.float64), mode="complete")
        A[c:, c + bk:] = (Qf.T @ A[c:, c + bk:].astype(np.float64)).astype(A.dtype)
        A[c:, c:c + bk] = 0
        A[c:c + bk, c:c + bk] = np.triu(R[:bk])
        n2 = n - c - bk
        if n2 > 0:
            Qf, R = np.linalg.qr(A[c:c + bk, c + bk:].T.astype(np.float64), mode="complete")
            A[c + bk:, c + bk:] = (A[c + bk:, c + bk:].astype(np.float64) @ Qf).astype(A.dtype)
            kk = min(bk, n2)
            A[c:c + bk, c + bk:] = 0
            A[c:c + bk, c + bk:c + bk + kk] = np.triu(R[:kk]).T[:bk, :kk] if n2 < bk else np.triu(R[:bk]).T
        c += bk


def blocked_columns(n: int, b: int, nb: int) -> int:
    """Columns reduced by the blocked path: whole blocks of nb full panels
    whose every row panel is at least b wide (n - k0 >= (nb + 1) b)."""
    k0 = 0
    while n - k0 >= (nb + 1) * b:
        k0 += nb * b
    return k0


def ge2band_blocked(A: np.ndarray, b: int, nb: int = 4) -> np.ndarray:
    A = np.array(A, copy=True)
    m, n = A.shape
    dt = A.dtype
    kend = blocked_columns(n, b, nb)
    k0 = 0
    while k0 < kend:
        V = np.zeros((m, 0), dt); Y = np.zeros((n, 0), dt)
        X = np.zeros((m, 0), dt); U = np.zeros((n, 0), dt)
        c = k0
        for _ in range(nb):
            P = A[c:, c:c + b] - V[c:] @ Y[c:c + b].T - X[c:] @ U[c:c + b].T
            Vj, Tj, Rj = cholqr_house(P)
            A[c:, c:c + b] = 0
            A[c:c + b, c:c + b] = Rj
            Vf = np.zeros((m, b), dt); Vf[c:] = Vj
            W = A[c:, c + b:].T @ Vj - Y[c + b:] @ (V[c:].T @ Vj) - U[c + b:] @ (X[c:].T @ Vj)
            Yf = np.zeros((n, b), dt); Yf[c + b:] = W @ Tj
            V = np.hstack([V, Vf]); Y = np.hstack([Y, Yf])
            Q = A[c:c + b, c + b:] - V[c:c + b] @ Y[c + b:].T - X[c:c + b] @ U[c + b:].T
            Uj, Sj, Lt = cholqr_house(Q.T)
            A[c:c + b, c + b:] = 0
            A[c:c + b, c + b:c + 2 * b] = Lt.T
            Uf = np.zeros((n, b), dt); Uf[c + b:] = Uj
            Z = A[c + b:, c + b:] @ Uj - V[c + b:] @ (Y[c + b:].T @ Uj) - X[c + b:] @ (U[c + b:].T @ Uj)
            Xf = np.zeros((m, b), dt); Xf[c + b:] = Z @ Sj
            X = np.hstack([X, Xf]); U = np.hstack([U, Uf])
            c += b
        k1 = c
        A[k1:, k1:] -= V[k1:] @ Y[k1:].T + X[k1:] @ U[k1:].T
        k0 = k1
    _tail_unblocked(A, kend, b)
    return A

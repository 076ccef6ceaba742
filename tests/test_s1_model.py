"""CPU checks of the blocked stage-1 model (tests/s1_model.py) -- the
executable specification of the GPU's delayed two-sided update -- against
the pinned oracle (svd_parallel.h:411 restated) and against exact linear
algebra.  No GPU."""
import numpy as np
import pytest

import s1_model as M
from oracle import oracle
from splitmix import uniform_matrix


def _band_mask(n, b):
    i, j = np.indices((n, n))
    return (j >= i) & (j - i <= b)


@pytest.mark.parametrize("n,b,nb", [(64, 4, 4), (256, 8, 4), (512, 32, 4), (512, 32, 2), (256, 16, 3)])
def test_model_matches_oracle_band(n, b, nb):
    A = uniform_matrix(n, seed=n + b, lo=1.0, hi=5.0)
    B = M.ge2band_blocked(A, b, nb)
    R = oracle.brd_p1(A, b)
    m = _band_mask(n, b)
    err = np.linalg.norm(np.abs(B[m]) - np.abs(R[m])) / np.linalg.norm(R[m])
    assert err < 1e-12, err
    assert np.all(B[~m] == 0)


@pytest.mark.parametrize("m,n,b", [(300, 300, 32), (333, 333, 7), (700, 420, 32)])
def test_model_preserves_singular_values(m, n, b):
    rng = np.random.default_rng(m + n + b)
    A = rng.standard_normal((m, n))
    B = M.ge2band_blocked(A, b, 4)
    i, j = np.indices((m, n))
    assert np.all(B[(j < i) | (j - i > b)] == 0)
    s = np.linalg.svd(A, compute_uv=False)
    t = np.linalg.svd(B, compute_uv=False)
    assert np.max(np.abs(s - t)) <= 1e-13 * s[0]


def test_cholqr_house_is_a_householder_block_reflector():
    rng = np.random.default_rng(5)
    P = rng.standard_normal((200, 32)) * 1e-170     # tiny entries: the power-of-two prescale
    V, T, R = M.cholqr_house(P)
    H = np.eye(200) - V @ T @ V.T
    assert np.allclose(H.T @ H, np.eye(200), atol=1e-14)
    HtP = H.T @ P
    assert np.allclose(HtP[:32], R, rtol=0, atol=1e-14 * np.abs(R).max())
    assert np.abs(HtP[32:]).max() <= 1e-14 * np.abs(R).max()
    assert np.allclose(np.diag(V[:32]), 1.0) and np.all(np.triu(V[:32], 1) == 0)

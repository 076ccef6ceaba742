"""Edge shapes through the C ABI (ragged and tiny
inputs, bands wider than the matrix, rectangular stage-1 inputs).

No reference output covers these shapes (the reference's tiled code needs
b | n and square inputs), so the checks are the reduction's own invariants
against numpy in fp64: exact zeros outside the band, the singular values of
the input preserved by stage 1, and stage 1 + sigma-preserving stage 2 +
brd_bdsvd reproducing them (|sigma_i - sigma_ref_i| <= tol * sigma_max:
fp64 1e-12 / 1e-11, fp32 2e-5 / 5e-5)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    import svdsolver_amd as S
    return S


def _outside(m, n, b):
    i, j = np.indices((m, n))
    return (j < i) | (j - i > b)


@pytest.mark.parametrize("T,tol1,tol2", [(np.float64, 1e-12, 1e-11), (np.float32, 2e-5, 5e-5)])
@pytest.mark.parametrize("n,b", [(1, 4), (2, 4), (3, 32), (17, 32), (31, 4), (32, 32), (33, 32), (65, 8),
                                 (100, 32), (257, 32), (513, 4), (1000, 32)])
def test_square_ragged_and_tiny(S, T, tol1, tol2, n, b):
    A = np.random.default_rng(n * 7 + b).uniform(1, 5, (n, n)).astype(T)
    ref = np.linalg.svd(A.astype(np.float64), compute_uv=False)
    band = S.brd_p1(A, b)
    assert np.all(band[_outside(n, n, b)] == 0)
    sb = np.linalg.svd(band.astype(np.float64), compute_uv=False)
    assert np.max(np.abs(sb - ref)) <= tol1 * ref[0]
    _, d, e = S.brd_p2(band, b, sigma=True)
    sv = S.bdsvd(d, e).astype(np.float64)
    assert np.max(np.abs(np.sort(sv)[::-1] - ref)) <= tol2 * ref[0]


@pytest.mark.parametrize("T,tol", [(np.float64, 1e-12), (np.float32, 2e-5)])
@pytest.mark.parametrize("m,n,b", [(300, 200, 32), (1025, 512, 32), (97, 40, 4), (64, 1, 4)])
def test_rectangular_stage1(S, T, tol, m, n, b):
    """m > n: the band sits in the top n x n block, every row below it is zero."""
    A = np.random.default_rng(m + n).uniform(1, 5, (m, n)).astype(T)
    ref = np.linalg.svd(A.astype(np.float64), compute_uv=False)
    band = S.brd_p1(A, b)
    assert np.all(band[_outside(m, n, b)] == 0)
    assert np.all(band[n:] == 0)
    sb = np.linalg.svd(band.astype(np.float64), compute_uv=False)
    assert np.max(np.abs(sb - ref)) <= tol * ref[0]

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


@pytest.mark.parametrize("T,scale,tol", [(np.float64, 2.0 ** -532, 1e-3), (np.float32, 2.0 ** -66, 1e-2),
                                         (np.float64, 2.0 ** 480, 1e-12)])
def test_extreme_scale_is_scale_invariant(S, T, scale, tol):
    """Entries near the ends of the exponent range (fp64 ~1e-160 / 1e144,
    fp32 ~1e-20).  The reflector scalars come from the hardware reciprocal
    (square root), which flushes denormal arguments to zero -- an infinite
    1/||x|| and NaN reflectors -- so the library prescales such arguments by a
    power of two.  At 1e-160 (fp64) and 1e-20 (fp32) the squared norms are
    themselves denormal (below 2^-1022 / 2^-126), where the arithmetic keeps
    fewer significant bits, as in the reference's unscaled sqrt(sum x^2)
    (svd_serial.h:189), so the check there is: finite, exact zeros outside
    the band, and s^-1 times the reduction of s A close to the reduction of A
    (tol 1e-3 / 1e-2); at 2^480 the squares stay normal and the reduction is
    scale-invariant to rounding (1e-12).  n = 300: the blocked stage 1 on the
    first 256 columns (blk_columns(300, 300, 32) = 256), the per-panel path after; stage 2 in the
    sigma-preserving geometry, compared through the singular values."""
    n, b = 300, 32
    A = np.random.default_rng(3).uniform(1, 5, (n, n)).astype(T)
    band = S.brd_p1(A, b).astype(np.float64)
    band_s0 = S.brd_p1((A * T(scale)).astype(T), b)
    assert np.all(band_s0[_outside(n, n, b)] == 0)
    band_s = band_s0.astype(np.float64) / scale
    assert np.all(np.isfinite(band_s))
    err = np.linalg.norm(np.abs(band_s) - np.abs(band)) / np.linalg.norm(band)
    assert err <= tol, err
    _, d, e = S.brd_p2(band.astype(T), b, sigma=True)
    _, d_s, e_s = S.brd_p2((band * scale).astype(T), b, sigma=True)
    assert np.all(np.isfinite(d_s)) and np.all(np.isfinite(e_s))
    sv = np.sort(S.bdsvd(d, e).astype(np.float64))
    sv_s = np.sort(S.bdsvd(d_s, e_s).astype(np.float64)) / scale
    assert np.all(np.isfinite(sv_s))
    assert np.max(np.abs(sv_s - sv)) <= 10 * tol * sv[-1], np.max(np.abs(sv_s - sv)) / sv[-1]


@pytest.mark.parametrize("kind", ["perm", "zero_cols", "rank1", "zero_col_in_panel", "dup_cols", "rank1_exact",
                                  "rank20_exact", "dup_rows"])
def test_structured_panels(S, kind):
    """Panels whose orthonormal factor has a permutation-like top block (the
    case the modified LU's sign choice exists for: with a fixed sign the
    reconstruction's W_t = Q_t - S would be singular), exactly zero panels,
    and rank-deficient inputs: a rank-1 matrix plus 1e-8 noise, and EXACTLY
    rank-deficient panels -- one zero column inside a non-zero
    panel, duplicated columns (and rows: the LQ side), an exact rank-1 outer
    product, an exact rank-20 product -- where the first CholeskyQR pass and
    then sCQR3's middle pass meet a zero pivot and the panel's basis is
    completed (cqr_shifted_pass).  Stage 1 (the blocked path: n = 512 reduces
    columns 0..383 blocked) must keep exact zeros outside the band and the
    input's singular values (fp64, 1e-12 sigma_max), and report no error."""
    n, b = 512, 32
    rng = np.random.default_rng(17)
    if kind == "perm":
        A = np.zeros((n, n))
        for k in range(0, n, b):
            A[k:k + b, k:k + b] = np.eye(b)[rng.permutation(b)]
        A += 1e-3 * rng.standard_normal((n, n))
    elif kind == "zero_cols":
        A = rng.uniform(1, 5, (n, n))
        A[:, :b] = 0.0
        A[:, 3 * b:5 * b] = 0.0
    elif kind == "rank1":
        A = np.outer(rng.standard_normal(n), rng.standard_normal(n)) + 1e-8 * rng.standard_normal((n, n))
    elif kind == "zero_col_in_panel":
        A = rng.uniform(1, 5, (n, n))
        A[:, 5] = 0.0
        A[:, 200] = 0.0
    elif kind == "dup_cols":
        A = rng.uniform(1, 5, (n, n))
        A[:, 7] = A[:, 3]
        A[:, 40] = A[:, 33]
        A[:, 300] = A[:, 290]
    elif kind == "dup_rows":
        A = rng.uniform(1, 5, (n, n))
        A[9] = A[2]
        A[100] = A[60]
    elif kind == "rank1_exact":
        A = np.outer(rng.standard_normal(n), rng.standard_normal(n))
    else:
        A = rng.standard_normal((n, 20)) @ rng.standard_normal((20, n))
    ref = np.linalg.svd(A, compute_uv=False)
    band = S.brd_p1(A, b)
    assert np.all(np.isfinite(band))
    assert np.all(band[_outside(n, n, b)] == 0)
    sb = np.linalg.svd(band, compute_uv=False)
    assert np.max(np.abs(sb - ref)) <= 1e-12 * ref[0], np.max(np.abs(sb - ref)) / ref[0]

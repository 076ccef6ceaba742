"""brd_bdsvd_* (host): singular values of an upper bidiagonal, the step after
stage 2 (replaces the reference's serial::qrd, svd_serial.h:368).  Checked
against numpy's LAPACK SVD of the same bidiagonal: absolute error
<= 1e-13 sigma_max (fp64), 1e-5 (fp32).  No GPU needed."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def B():
    import svdsolver_amd.brd as B
    return B


def _ref(d, e):
    n = len(d)
    M = np.diag(np.asarray(d, np.float64))
    if n > 1:
        M += np.diag(np.asarray(e, np.float64), 1)
    return np.linalg.svd(M, compute_uv=False)


@pytest.mark.parametrize("n", [1, 2, 3, 17, 400, 1500])
def test_random_f64(B, n):
    rng = np.random.default_rng(n)
    d, e = rng.uniform(-3, 3, n), rng.uniform(-3, 3, max(n - 1, 0))
    ref = _ref(d, e)
    assert np.max(np.abs(B.bdsvd(d, e) - ref)) <= 1e-13 * ref[0]


def test_zero_and_tiny_entries(B):
    d = np.array([1e-30, 2.0, 0.0, 3.0, 1e-300, 5.0, 0.0])
    e = np.array([1.0, 0.0, 2.0, 1e-20, 4.0, 0.0])
    ref = _ref(d, e)
    assert np.max(np.abs(B.bdsvd(d, e) - ref)) <= 1e-13 * ref[0]


def test_graded(B):
    d, e = np.logspace(0, -15, 200), np.logspace(-1, -16, 199)
    ref = _ref(d, e)
    assert np.max(np.abs(B.bdsvd(d, e) - ref)) <= 1e-13 * ref[0]


def test_descending_and_nonnegative(B):
    rng = np.random.default_rng(7)
    sv = B.bdsvd(rng.standard_normal(64), rng.standard_normal(63))
    assert np.all(sv >= 0) and np.all(np.diff(sv) <= 0)


def test_f32(B):
    rng = np.random.default_rng(9)
    d = rng.uniform(1, 2, 300).astype(np.float32)
    e = rng.uniform(1, 2, 299).astype(np.float32)
    sv = B.bdsvd(d, e)
    assert sv.dtype == np.float32
    ref = _ref(d, e)
    assert np.max(np.abs(sv - ref)) <= 1e-5 * ref[0]


def test_rejects_non_finite(B):
    with pytest.raises(B.BrdError):
        B.bdsvd(np.array([1.0, np.nan]), np.array([1.0]))

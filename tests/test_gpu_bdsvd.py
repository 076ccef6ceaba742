"""Bidiagonal singular values on the GPU (brd_bdsvd_dev_*, svdsolver_amd.bdsvd_gpu;
SURVEY.md 8(f) rank 2 "on host/GPU").  Checked against the library's host
Golub-Kahan QR (brd_bdsvd_*, itself checked against numpy in test_bdsvd.py)
and against numpy's dense SVD, with absolute tolerances in units of sigma_max
(the accuracy both methods promise): fp64 1e-13, fp32 2e-6 against an fp64
reference of the same (rounded) input."""
import time

import numpy as np
import pytest

import svdsolver_amd as S

pytestmark = pytest.mark.gpu


def _dense(d, e):
    n = d.shape[0]
    B = np.diag(d.astype(np.float64))
    if n > 1:
        B += np.diag(e.astype(np.float64), 1)
    return B


def _gpu(d, e):
    import torch
    td = torch.from_numpy(np.ascontiguousarray(d)).cuda()
    te = torch.from_numpy(np.ascontiguousarray(e if e.size else np.zeros(0, d.dtype))).cuda()
    return S.bdsvd_gpu(td, te).cpu().numpy()


@pytest.mark.parametrize("n", [1, 2, 3, 17, 300, 1500])
def test_random_bidiagonal_matches_host_qr(n):
    rng = np.random.default_rng(100 + n)
    d = rng.uniform(-3, 3, n)
    e = rng.uniform(-3, 3, max(n - 1, 0))
    got = _gpu(d, e)
    ref = S.bdsvd(d, e)
    assert np.all(np.diff(got) <= 0), "descending order"
    assert np.max(np.abs(got - ref)) <= 1e-13 * ref[0]


def test_graded_and_zero_entries_match_numpy():
    """Entries over ten decades, exact zeros on both diagonals (split and
    zero singular values): numpy's dense SVD as the reference."""
    rng = np.random.default_rng(7)
    n = 200
    d = 10.0 ** (-np.linspace(0, 10, n)) * rng.uniform(0.5, 1.5, n)
    e = 10.0 ** (-np.linspace(0, 10, n - 1)) * rng.uniform(0.5, 1.5, n - 1)
    d[[5, 60, 61, 150]] = 0.0
    e[[10, 11, 90]] = 0.0
    got = _gpu(d, e)
    ref = np.linalg.svd(_dense(d, e), compute_uv=False)
    assert np.max(np.abs(got - ref)) <= 1e-13 * ref[0]
    assert got[-1] <= 1e-13 * ref[0]   # d has zeros: B is singular


def test_fp32_against_fp64_reference():
    rng = np.random.default_rng(11)
    n = 500
    d = rng.uniform(0.1, 2, n).astype(np.float32)
    e = rng.uniform(0.1, 2, n - 1).astype(np.float32)
    got = _gpu(d, e).astype(np.float64)
    ref = S.bdsvd(d.astype(np.float64), e.astype(np.float64))
    assert np.max(np.abs(got - ref)) <= 2e-6 * ref[0]


def test_singular_values_gpu_pipeline_matches_numpy():
    """Stage 1 + sigma-preserving stage 2 + GPU bidiagonal values, all on the
    GPU: numpy's singular values of the dense input."""
    import torch
    rng = np.random.default_rng(13)
    n = 1024
    A = rng.uniform(0, 5, (n, n))
    got = S.singular_values_gpu(torch.from_numpy(A).cuda()).cpu().numpy()
    ref = np.linalg.svd(A, compute_uv=False)
    assert np.max(np.abs(got - ref)) <= 1e-12 * ref[0]


def test_bench_size_bidiagonal_against_host():
    """n = 8192 (the bench size): the GPU values against the host QR, and the
    GPU call is faster than the host one."""
    import torch
    rng = np.random.default_rng(17)
    n = 8192
    d = rng.uniform(-2, 2, n)
    e = rng.uniform(-2, 2, n - 1)
    td, te = torch.from_numpy(d).cuda(), torch.from_numpy(e).cuda()
    S.bdsvd_gpu(td, te)   # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = S.bdsvd_gpu(td, te).cpu().numpy()
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref = S.bdsvd(d, e)
    t_host = time.perf_counter() - t0
    assert np.max(np.abs(got - ref)) <= 1e-13 * ref[0]
    print(f"bdsvd n={n}: GPU {t_gpu * 1e3:.1f} ms, host {t_host * 1e3:.1f} ms")
    assert t_gpu < t_host

"""GPU correctness at the sizes bench.py measures (BASELINE.json configs[2..4]):
8192^2 fp64, 8192^2 fp32 and 16384^2 fp64, band 32, each a full two-stage
reduction through the C ABI, plus run-twice determinism.

At these sizes no reference output exists (the reference's own CPU code would
need ~45 min at 8192), so the checks are the
size-independent properties of the reduction:

* stage 1 leaves EXACT zeros outside the band (diagonals 0..b);
* stage 1 is orthogonal: ||band||_F = ||A||_F (fp64 <= 1e-13, fp32 <= 1e-5);
* stage 1 + sigma-preserving stage 2 (BRD_SIGMA) + brd_bdsvd give the
  singular values of A: fp64 against an independent fp64 eigensolver on A^T A
  (torch.linalg.eigvalsh, rocSOLVER): |sigma_i^2 - lambda_i| <= 1e-11 sigma_max^2
  (the eigensolver's own error is ~n eps sigma_max^2, 2e-12 at n = 16384);
  fp32 against the same fp64 reference, |sigma_i - sqrt(lambda_i)| <= 2e-5 sigma_max;
* the reference-geometry (compat) stage 2 -- the path the benchmark times --
  finishes with its sticky stall word clear and a finite bidiagonal;
* no stage-2 stall word is left set (brd_check_errors).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B = 32


@pytest.fixture(scope="module")
def S():
    import svdsolver_amd as S
    return S


def _rand(n, dtype, seed):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand((n, n), dtype=dtype, device="cuda", generator=g) * 5.0


def _outside_band_nonzeros(M, b):
    import torch
    n = M.shape[0]
    bad = 0
    for r0 in range(0, n, 2048):        # row blocks: bounded temporaries at 16384
        blk = M[r0:r0 + 2048]
        i = torch.arange(r0, r0 + blk.shape[0], device=M.device)[:, None]
        j = torch.arange(n, device=M.device)[None, :]
        out = (j < i) | (j - i > b)
        bad += int(torch.count_nonzero(blk[out]))
    return bad


def _gram_eigs(A64):
    """Eigenvalues of A^T A (fp64, ascending -> returned descending)."""
    import torch
    G = A64.T @ A64
    lam = torch.linalg.eigvalsh(G)
    del G
    return torch.flip(lam, [0]).cpu().numpy()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,tname", [(8192, "f64"), (8192, "f32"), (16384, "f64")])
def test_two_stage_at_bench_size(S, n, tname):
    import torch
    dt = torch.float64 if tname == "f64" else torch.float32
    A = _rand(n, dt, seed=n + (1 if tname == "f32" else 0))
    A64 = A.to(torch.float64)
    fa = float(torch.linalg.norm(A64))

    band = A.clone()
    S.ge2band(band, B)
    assert _outside_band_nonzeros(band, B) == 0, "stage 1 left nonzeros outside the band"
    fb = float(torch.linalg.norm(band.to(torch.float64)))
    assert abs(fa - fb) / fa <= (1e-13 if tname == "f64" else 1e-5), (fa, fb)

    # sigma-preserving stage 2 + host bidiagonal QR -> singular values
    work = band.clone()
    d, e = S.band2bd(work, B, sigma=True)
    S.check_errors()
    sv = S.bdsvd(d, e).astype(np.float64)
    del work
    lam = np.clip(_gram_eigs(A64), 0.0, None)
    del A64
    smax2 = lam[0]
    if tname == "f64":
        err = np.max(np.abs(sv ** 2 - lam)) / smax2
        assert err <= 1e-11, err
    else:
        err = np.max(np.abs(sv - np.sqrt(lam))) / np.sqrt(smax2)
        assert err <= 2e-5, err

    # the benchmark's stage 2: the reference's window geometry
    d, e = S.band2bd(band, B)
    S.check_errors()
    assert bool(torch.isfinite(d).all()) and bool(torch.isfinite(e).all())
    assert float(torch.abs(d).max()) > 0


def _bd_err(d, e, d0, e0):
    import torch
    got = torch.cat([d.abs(), e.abs()]).double()
    ref = torch.cat([d0.abs(), e0.abs()]).double()
    return float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,tname", [(8192, "f64"), (8192, "f32"), (16384, "f64")])
def test_compat_stage2_within_envelope_at_bench_size(S, n, tname):
    """The stage 2 every bench line times (the reference's window geometry,
    fast arithmetic) against the GPU exact-order sweep on the same band -- the
    exact-order sweep is bit-identical to svd_parallel.h:640-695's operation
    order (tests/test_gpu_parity.py pins it to the fixtures).  The compat
    geometry is ill-conditioned (Stage 2), so the bound is the
    reference's own sensitivity: how far its exact-order output moves when
    the band is perturbed by one rounding error per element (two trials),
    times 10, as in test_gpu_parity.py::_envelope."""
    import torch
    dt = torch.float64 if tname == "f64" else torch.float32
    A = _rand(n, dt, seed=3 * n + (1 if tname == "f32" else 0))
    S.ge2band(A, B)
    band = A
    del A
    eps = float(torch.finfo(dt).eps)

    def sweep(M, exact):
        W = M.clone()
        d, e = S.band2bd(W, B, exact_order=exact)
        S.check_errors()
        del W
        return d.clone(), e.clone()

    d0, e0 = sweep(band, True)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    env = 0.0
    for _ in range(2):
        p = band * (1 + eps * torch.randn(band.shape, dtype=dt, device="cuda", generator=g))
        d1, e1 = sweep(p, True)
        del p
        env = max(env, _bd_err(d1, e1, d0, e0))
    d, e = sweep(band, False)
    assert bool(torch.isfinite(d).all()) and bool(torch.isfinite(e).all())
    err = _bd_err(d, e, d0, e0)
    assert env > 0
    assert err <= 10 * env + 10 * eps, (err, env)


@pytest.mark.parametrize("n", [1024, 8192])
def test_two_stage_bitwise_reproducible(S, n):
    """Run twice, bitwise equal ('race detection'): stage 1
    sums its cross-wave partials in a fixed order, stage 2's sweeps follow the
    lag-3 schedule in a fixed arithmetic order, so the band and the bidiagonal
    do not depend on scheduling."""
    import torch
    A = _rand(n, torch.float64, seed=77)
    outs = []
    for _ in range(2):
        M = A.clone()
        S.ge2band(M, B)
        band = M.clone()
        d, e = S.band2bd(M, B)
        outs.append((band, d, e))
    assert torch.equal(outs[0][0], outs[1][0]), "stage 1 output differs between two runs"
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2]), "stage 2 output differs"


@pytest.mark.parametrize("n,T", [(8192, "float64"), (4096, "float64"), (8192, "float32")])
def test_stage1_bitwise_over_many_runs(S, n, T):
    """Stage 1 run eight times on the same matrix gives the same band bit for
    bit (round 4: a counted wait in k_blkupd_p that was too loose on a
    workgroup's first tile let a chunk's DMAs still be in flight when it was
    read -- about one run pair in fourteen differed at N = 8192; a two-run
    test catches that rarely, eight runs make a recurrence likely to show)."""
    import torch
    dt = getattr(torch, T)
    g = torch.Generator(device="cuda")
    g.manual_seed(77)
    A = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
    ref = None
    for r in range(8):
        M = A.clone()
        S.ge2band(M, B)
        if ref is None:
            ref = M
        else:
            assert torch.equal(ref, M), f"run {r} differs from run 0"

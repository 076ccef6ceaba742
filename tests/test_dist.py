"""Multi-GPU stage 1 (block-cyclic column shards, svdsolver_amd/csrc/brd_dist.hip).

CPU (gloo, world size 2 and 3): the layout helpers against the library's
brd_dist_local_cols, and the distributed algorithm itself -- its numpy
restatement tests/dist_sim.py, run as separate processes with the library's
collectives through torch.distributed -- against the CPU oracle (|band|,
the band is unique up to signs; fp64 normwise <= 1e-12).

GPU: the library's distributed path with 2 and 3 ranks sharing cuda:0 through
the host-callback communicator (gloo), and with RCCL at world size 1, against
the single-GPU stage 1 (fp64 <= 1e-12, fp32 <= 1e-4 normwise on |band|) --
RCCL cannot put two ranks on one GPU, so multi-rank RCCL runs only on a
multi-GPU node (bench.py --gpus N).
"""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _band_mask(n, b):
    i, j = np.indices((n, n))
    return (j >= i) & (j - i <= b)


def _band_err(a, ref, b):
    m = _band_mask(a.shape[0], b)
    da = np.abs(a[m]).astype(np.float64) - np.abs(ref[m]).astype(np.float64)
    return float(np.linalg.norm(da) / np.linalg.norm(ref[m].astype(np.float64)))


# ---------------------------------------------------------------------------
# layout (CPU)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n,b", [(64, 8), (100, 32), (1000, 32), (33, 32), (8192, 32)])
@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_local_cols_match_library(n, b, P):
    from svdsolver_amd import dist, lib
    tot = 0
    for r in range(P):
        nl = dist.local_cols(n, b, P, r)
        assert nl == lib.brd_dist_local_cols(n, b, P, r)
        assert nl == len(dist.global_columns(n, b, P, r))
        tot += nl
    assert tot == n


def test_shard_roundtrip():
    from svdsolver_amd import dist
    rng = np.random.default_rng(0)
    A = rng.standard_normal((70, 70))
    for P in (1, 2, 3):
        parts = [dist.shard(A, 8, P, r) for r in range(P)]
        assert np.array_equal(dist.unshard(parts, 70, 8), A)


# ---------------------------------------------------------------------------
# the algorithm on CPU (gloo, separate processes)
# ---------------------------------------------------------------------------
def _sim_worker(rank, world, port, n, b, seed, out_path):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as tdist
    import dist_sim
    from svdsolver_amd import dist
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(seed)
    A = rng.uniform(1, 5, (n, n))
    loc = dist.shard(A, b, world, rank).astype(np.float64)
    dist_sim.ge2band_dist_sim(loc, n, b, rank, world, tdist)
    import torch
    wmax = max(dist.local_cols(n, b, world, r) for r in range(world))
    mine = np.zeros((n, wmax))
    mine[:, :loc.shape[1]] = loc
    parts = [torch.zeros((n, wmax), dtype=torch.float64) for _ in range(world)]
    tdist.all_gather(parts, torch.from_numpy(mine))
    if rank == 0:
        shards = [parts[r].numpy()[:, :dist.local_cols(n, b, world, r)] for r in range(world)]
        np.save(out_path, dist.unshard(shards, n, b))
    tdist.barrier()
    tdist.destroy_process_group()


def _blk_sim_worker(rank, world, port, n, b, seed, out_path):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as tdist
    import dist_blk_sim
    from svdsolver_amd import dist
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    A = np.random.default_rng(seed).uniform(1, 5, (n, n))
    loc = dist.shard(A, b, world, rank).astype(np.float64)
    dist_blk_sim.ge2band_blk_dist_sim(loc, n, b, rank, world, tdist)
    wmax = max(dist.local_cols(n, b, world, r) for r in range(world))
    mine = np.zeros((n, wmax))
    mine[:, :loc.shape[1]] = loc
    parts = [torch.zeros((n, wmax), dtype=torch.float64) for _ in range(world)]
    tdist.all_gather(parts, torch.from_numpy(mine))
    if rank == 0:
        shards = [parts[r].numpy()[:, :dist.local_cols(n, b, world, r)] for r in range(world)]
        np.save(out_path, dist.unshard(shards, n, b))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 512), (3, 600), (4, 704), (8, 640)])
def test_blocked_distributed_algorithm_gloo(world, n, tmp_path):
    """The blocked distributed stage 1's data flow (tests/dist_blk_sim.py:
    owner-side column-panel QR + broadcast, local Y pass, gathered row panel
    factored on every rank, all-reduced X pass, local block update; b = 32,
    blocks of 4 panels, the per-panel tail after) on 2-4 gloo ranks: the band
    matches the single-process blocked model (tests/s1_model.py) in |.| and
    keeps the singular values (fp64, 1e-12)."""
    import torch.multiprocessing as mp
    import s1_model
    b = 32
    out = str(tmp_path / "band.npy")
    mp.spawn(_blk_sim_worker, args=(world, _free_port(), n, b, 11, out), nprocs=world, join=True)
    band = np.load(out)
    A = np.random.default_rng(11).uniform(1, 5, (n, n))
    ref = s1_model.ge2band_blocked(A, b)
    assert _band_err(band, ref, b) <= 1e-12
    assert np.all(np.abs(band[~_band_mask(n, b)]) < 1e-12 * np.abs(ref).max())
    sa, sb = np.linalg.svd(A, compute_uv=False), np.linalg.svd(band, compute_uv=False)
    assert np.max(np.abs(sa - sb)) <= 1e-12 * sa[0]


@pytest.mark.parametrize("world,n,b", [(2, 96, 8), (3, 100, 8), (2, 130, 32)])
def test_distributed_algorithm_gloo(world, n, b, tmp_path):
    import torch.multiprocessing as mp
    from oracle import oracle
    out = str(tmp_path / "band.npy")
    mp.spawn(_sim_worker, args=(world, _free_port(), n, b, 3, out), nprocs=world, join=True)
    band = np.load(out)
    A = np.random.default_rng(3).uniform(1, 5, (n, n))
    if n % b == 0:
        ref = oracle.brd_p1(A, b)          # the reference's tiled algorithm needs b | n
    else:
        import dist_sim
        ref = dist_sim.ge2band_dist_sim(A.copy(), n, b, 0, 1, dist_sim.LocalComm)
    assert _band_err(band, ref, b) <= 1e-12
    assert np.all(np.abs(band[~_band_mask(n, b)]) < 1e-12 * np.abs(ref).max())
    # size-independent: the two-sided orthogonal reduction keeps the singular values
    sa, sb = np.linalg.svd(A, compute_uv=False), np.linalg.svd(band, compute_uv=False)
    assert np.max(np.abs(sa - sb)) <= 1e-12 * sa[0]


# ---------------------------------------------------------------------------
# the library's distributed path on the GPU
# ---------------------------------------------------------------------------
def _gpu_worker(rank, world, port, n, b, dtype, mode, out_path, root=0):
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as tdist
    from svdsolver_amd import dist
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    if mode == "rccl":
        dist.init_rccl()
    else:
        dist.init_host()
    rng = np.random.default_rng(5)
    A = rng.uniform(1, 5, (n, n)).astype(dtype)
    loc = torch.from_numpy(dist.shard(A, b, world, rank)).cuda()
    dist.ge2band(loc, n, b)
    B = dist.gather_band(loc, n, b, root=root)
    if rank == root:
        np.save(out_path, B.cpu().numpy())
    else:
        assert B is None
    dist.finalize()
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,b,dtype,mode", [
    (2, 640, 32, np.float64, "host"),
    (3, 600, 32, np.float64, "host"),     # ragged last panel (600 = 18 * 32 + 24)
    (2, 512, 16, np.float32, "host"),
    (1, 512, 32, np.float64, "rccl"),
    # the blocked distributed path over >= 5 panels: 2 blocks of
    # 4 panels at 1024, 8 at 1100 with a ragged tail, 4 ranks
    (2, 1024, 32, np.float64, "host"),
    (3, 1100, 32, np.float64, "host"),
    (4, 1024, 32, np.float64, "host"),
    (1, 1024, 32, np.float64, "rccl"),
    # the P = 8 layout of configs[4]: 8 ranks on the blocked
    # path with the sharded row-panel CholeskyQR, and a ragged tail
    (8, 2048, 32, np.float64, "host"),
    (8, 2096, 32, np.float64, "host"),
])
def test_distributed_stage1_gpu(world, n, b, dtype, mode, tmp_path):
    """Against the single-GPU stage 1 (|band|, fp64 1e-12): with b = 32 in
    fp64 the columns the blocked path covers (blk_columns) run the blocked
    distributed form (brd_stage1_blk.hip blk_ge2band_dist), the rest the
    per-panel distributed loop."""
    import torch.multiprocessing as mp
    import svdsolver_amd as S
    out = str(tmp_path / "band.npy")
    mp.spawn(_gpu_worker, args=(world, _free_port(), n, b, dtype, mode, out), nprocs=world, join=True)
    band = np.load(out)
    A = np.random.default_rng(5).uniform(1, 5, (n, n)).astype(dtype)
    ref = S.brd_p1(A.astype(np.float64), b)
    tol = 1e-12 if dtype == np.float64 else 1e-4
    assert _band_err(band, ref, b) <= tol
    assert np.all(band[~_band_mask(n, b)] == 0)


@pytest.mark.gpu
def test_distributed_gather_band_to_last_rank(tmp_path):
    """The band gathered on a rank other than 0 (bench.py's pipelined multi-GPU
    mode sends matrix j's band to rank j mod P): 3 ranks, root 2."""
    import torch.multiprocessing as mp
    import svdsolver_amd as S
    out = str(tmp_path / "band.npy")
    n, b = 600, 32
    mp.spawn(_gpu_worker, args=(3, _free_port(), n, b, np.float64, "host", out, 2), nprocs=3, join=True)
    band = np.load(out)
    A = np.random.default_rng(5).uniform(1, 5, (n, n))
    ref = S.brd_p1(A, b)
    assert _band_err(band, ref, b) <= 1e-12
    assert np.all(band[~_band_mask(n, b)] == 0)


def _band_part(X, b):
    """Diagonals 0..b of a torch matrix, zeros elsewhere."""
    import torch
    return torch.triu(X) - torch.triu(X, diagonal=b + 1)


def _gpu_worker_full_size(rank, world, port, n, b, out_path):
    """configs[4]'s layout at its size: every rank draws the same matrix on the
    GPU (seeded), keeps its block-cyclic column shard, runs the distributed
    stage 1, and the band is gathered on rank 0, which compares it on the GPU
    with the one-GPU stage 1 of the same matrix (only the numbers leave HBM)."""
    sys.path.insert(0, os.path.dirname(HERE))
    import json
    import torch
    import torch.distributed as tdist
    import svdsolver_amd as S
    from svdsolver_amd import dist
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dist.init_host()

    def draw():
        g = torch.Generator(device="cuda")
        g.manual_seed(16384)
        return torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) * 5.0

    A = draw()
    loc = dist.shard(A, b, world, rank)
    del A
    torch.cuda.empty_cache()
    dist.ge2band(loc, n, b)
    B = dist.gather_band(loc, n, b, root=0)
    del loc
    if rank == 0:
        R = draw()
        S.ge2band(R, b)
        Bb, Rb = _band_part(B, b), _band_part(R, b)
        out = {"err": float(torch.linalg.norm(Bb.abs() - Rb.abs()) / torch.linalg.norm(Rb)),
               "outside_nonzeros": int(torch.count_nonzero(B - Bb)),
               "finite": bool(torch.isfinite(Bb).all()),
               "sign_diffs": int(torch.count_nonzero((torch.sign(Bb) != torch.sign(Rb)) & (Rb.abs() > 1e-9 * Rb.abs().max())))}
        with open(out_path, "w") as f:
            json.dump(out, f)
    dist.finalize()
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_distributed_stage1_p8_at_configs4_size(tmp_path):
    """configs[4]'s P = 8 block-column layout at its real size
    (n = 16384 fp64, b = 32: 2048 local columns per rank, the blocked path with
    the sharded row-panel CholeskyQR over 508 panels and the per-panel tail),
    8 ranks sharing cuda:0 through the host-callback communicator (RCCL cannot
    put two ranks on one GPU).  The gathered band against the one-GPU stage 1:
    |band| normwise <= 1e-12, exact zeros outside the band.  Reference
    decomposition: svd_parallel.h:477-485 (the tile-column loop)."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "p8.json")
    mp.spawn(_gpu_worker_full_size, args=(8, _free_port(), 16384, 32, out), nprocs=8, join=True)
    r = json.load(open(out))
    print(r)
    assert r["finite"]
    assert r["err"] <= 1e-12, r
    assert r["outside_nonzeros"] == 0, r


def _gpu_lanes_worker(rank, world, port, n, b, mode, lanes, out_path):
    """One communicator per stream (brd_dist_init binds it to the library's
    current stream): `lanes` matrices reduced at once, each on its own stream
    with its own communicator and workspace."""
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as tdist
    from svdsolver_amd import dist
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    streams = [torch.cuda.Stream() for _ in range(lanes)]
    for s in streams:
        if mode == "rccl":
            dist.init_rccl(stream=s)
        else:
            dist.init_host(stream=s)
    locs, outs = [], []
    for k, s in enumerate(streams):
        A = np.random.default_rng(10 + k).uniform(1, 5, (n, n))
        loc = torch.from_numpy(dist.shard(A, b, world, rank)).cuda()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            dist.ge2band(loc, n, b, sync=False)
            outs.append(dist.gather_band(loc, n, b, root=0, sync=False))
        locs.append(loc)
    torch.cuda.synchronize()
    if rank == 0:
        np.save(out_path, np.stack([B.cpu().numpy() for B in outs]))
    dist.finalize()
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,lanes", [(1, "rccl", 3), (2, "host", 2)])
def test_distributed_stage1_streams_with_own_communicators(world, mode, lanes, tmp_path):
    import torch.multiprocessing as mp
    import svdsolver_amd as S
    out = str(tmp_path / "bands.npy")
    n, b = 512, 32
    mp.spawn(_gpu_lanes_worker, args=(world, _free_port(), n, b, mode, lanes, out), nprocs=world, join=True)
    bands = np.load(out)
    for k in range(lanes):
        A = np.random.default_rng(10 + k).uniform(1, 5, (n, n))
        ref = S.brd_p1(A, b)
        assert _band_err(bands[k], ref, b) <= 1e-12, k
        assert np.all(bands[k][~_band_mask(n, b)] == 0)


def _edge_matrix(kind, n, b):
    rng = np.random.default_rng(17)
    if kind == "rank1_exact":
        return np.outer(rng.standard_normal(n), rng.standard_normal(n))
    if kind == "rank20_exact":
        return rng.standard_normal((n, 20)) @ rng.standard_normal((20, n))
    A = rng.uniform(1, 5, (n, n))
    if kind == "dup_rows":      # the row panels' (LQ side) duplicated columns
        A[9] = A[2]
        A[100] = A[60]
    elif kind == "zero_col_in_panel":
        A[:, 5] = 0.0
        A[:, 200] = 0.0
    return A


def _edge_worker(rank, world, port, n, b, kind, out_path):
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as tdist
    from svdsolver_amd import dist
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dist.init_host()
    A = _edge_matrix(kind, n, b)
    loc = torch.from_numpy(dist.shard(A, b, world, rank)).cuda()
    dist.ge2band(loc, n, b)
    B = dist.gather_band(loc, n, b, root=0)
    if rank == 0:
        np.save(out_path, B.cpu().numpy())
    dist.finalize()
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,n", [(2, 512), (3, 512), (8, 2048)])
@pytest.mark.parametrize("kind", ["rank1_exact", "rank20_exact", "dup_rows", "zero_col_in_panel"])
def test_distributed_structured_panels(world, n, kind, tmp_path):
    """Exactly rank-deficient row panels on the sharded CholeskyQR (ADVICE r4:
    the completion vectors of sCQR3's middle pass, k_cqr_mid, must keep the
    transform orthogonal when the panel's rows are spread over ranks): the
    gathered band keeps exact zeros outside it and the input's singular
    values (fp64, 1e-12 sigma_max), as on one GPU (test_gpu_edges.py).  At
    P = 8, n = 2048 the deficient panels' single CholeskyQR pass
    on the completed y (one pass where cqr_shifted_pass makes two) runs over
    rows spread across 8 ranks and 508..32 rows each: a transform off
    orthogonality by more than ~1e-12 would show in the singular values."""
    import torch.multiprocessing as mp
    b = 32
    out = str(tmp_path / "band.npy")
    mp.spawn(_edge_worker, args=(world, _free_port(), n, b, kind, out), nprocs=world, join=True)
    band = np.load(out)
    A = _edge_matrix(kind, n, b)
    ref = np.linalg.svd(A, compute_uv=False)
    assert np.all(np.isfinite(band))
    assert np.all(band[~_band_mask(n, b)] == 0)
    sb = np.linalg.svd(band, compute_uv=False)
    assert np.max(np.abs(sb - ref)) <= 1e-12 * ref[0], np.max(np.abs(sb - ref)) / ref[0]

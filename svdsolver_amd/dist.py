"""Multi-GPU stage 1: one process per GPU, block-cyclic column shards.

Layout (include/brd.h, brd_dist_*): global column panel ``p`` (columns
``[p*b, p*b + b)``) lives on rank ``p % P`` as its local panel ``p // P``; a
rank's shard is the ``m x n_loc`` row-major matrix of its columns in device
memory.  The panel loop itself runs in the library (brd_dist.hip): per panel
one broadcast of the column panel, one all-gather of the ranks' b x b R
factors and one all-reduce of the root's b x m projection.

Communicators:

* :func:`init_rccl` -- RCCL over xGMI (production).  Rank 0 draws the unique
  id (``brd_dist_unique_id``) and shares it through ``torch.distributed``.
* :func:`init_host` -- collectives through a host callback that runs them
  with ``torch.distributed`` (any backend, e.g. gloo).  Used where RCCL cannot
  run (several ranks on one GPU in tests).

The reference has no multi-GPU path; this is new API.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np

from .brd import (BRD_ASYNC, BRD_DEVICE_PTR, COLL_FN, _bind_stream, _check, _row_stride, _sfx, lib)

COLL_BCAST, COLL_ALLGATHER, COLL_ALLREDUCE_SUM = 0, 1, 2
DT_BYTE, DT_F32, DT_F64 = 0, 1, 2

_keep = []   # ctypes callbacks / closures that must outlive the communicator


# ---------------------------------------------------------------------------
# layout (pure Python; brd_dist_local_cols is the library's twin)
# ---------------------------------------------------------------------------
def npanels(n: int, b: int) -> int:
    return (n + b - 1) // b


def panel_owner(p: int, nranks: int) -> int:
    return p % nranks


def local_cols(n: int, b: int, nranks: int, rank: int) -> int:
    """Columns of rank ``rank``'s shard."""
    return sum(min(b, n - p * b) for p in range(rank, npanels(n, b), nranks))


def global_columns(n: int, b: int, nranks: int, rank: int) -> np.ndarray:
    """Global column index of each local column of ``rank`` (in local order)."""
    cols = [np.arange(p * b, min(n, p * b + b)) for p in range(rank, npanels(n, b), nranks)]
    return np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)


def shard(A, b: int, nranks: int, rank: int):
    """This rank's column shard of a full matrix (numpy array or torch tensor),
    contiguous."""
    cols = global_columns(A.shape[1], b, nranks, rank)
    if type(A).__module__.startswith("torch"):
        import torch
        return A[:, torch.as_tensor(cols, device=A.device, dtype=torch.long)].contiguous()
    return np.ascontiguousarray(A[:, cols])


def unshard(shards: List, n: int, b: int):
    """Inverse of :func:`shard` (numpy), for tests."""
    P = len(shards)
    m = shards[0].shape[0]
    out = np.zeros((m, n), dtype=shards[0].dtype)
    for r, S in enumerate(shards):
        out[:, global_columns(n, b, P, r)] = S
    return out


# ---------------------------------------------------------------------------
# communicators
# ---------------------------------------------------------------------------
def _bind(stream) -> None:
    if stream is not None:
        _check("brd_set_stream", lib.brd_set_stream(ctypes.c_void_p(stream.cuda_stream)))


def init_rccl(group=None, stream=None) -> None:
    """RCCL communicator over the processes of ``group`` (torch.distributed
    must be initialised; each process has selected its GPU).  With ``stream``
    (a torch CUDA stream) the communicator serves the calls made on that
    stream only (one communicator per stream lets several matrices' reductions
    run at once); the first communicator is also the default."""
    import torch.distributed as dist
    _bind(stream)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    buf = ctypes.create_string_buffer(128)
    obj = [None]
    if rank == 0:
        _check("brd_dist_unique_id", lib.brd_dist_unique_id(buf, 128))
        obj = [bytes(buf.raw)]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    idb = ctypes.create_string_buffer(obj[0], 128)
    _check("brd_dist_init", lib.brd_dist_init(rank, world, idb, 128))


class _DevArray:
    """A raw device pointer as a 1-D array (``__cuda_array_interface__``)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


_TYPESTR = {DT_BYTE: "|u1", DT_F32: "<f4", DT_F64: "<f8"}


def init_host(group=None, stream=None) -> None:
    """Host-callback communicator: the library drains its stream and calls
    back; the collective runs through ``torch.distributed`` on host copies of
    the device buffers (works with gloo, several ranks per GPU).  ``stream``:
    as in :func:`init_rccl`."""
    import torch
    import torch.distributed as dist
    _bind(stream)
    rank, world = dist.get_rank(group), dist.get_world_size(group)

    def dev(ptr, count, dtype):
        return torch.as_tensor(_DevArray(ptr, count, _TYPESTR[dtype]), device="cuda")

    def coll(op, send, recv, count, dtype, root, _user):
        try:
            if op == COLL_BCAST:
                d = dev(recv, count, dtype)
                h = d.cpu()
                dist.broadcast(h, src=dist.get_global_rank(group, root) if group is not None else root, group=group)
                d.copy_(h)
            elif op == COLL_ALLGATHER:
                s = dev(send, count, dtype).cpu()
                d = dev(recv, count * world, dtype)
                parts = [torch.empty_like(s) for _ in range(world)]
                dist.all_gather(parts, s, group=group)
                d.copy_(torch.cat(parts))
            elif op == COLL_ALLREDUCE_SUM:
                d = dev(recv, count, dtype)
                h = d.cpu()
                dist.all_reduce(h, group=group)
                d.copy_(h)
            else:
                return 1
            torch.cuda.synchronize()
            return 0
        except Exception as exc:   # report through the C return code
            print(f"[svdsolver_amd.dist] collective {op} failed: {exc}")
            return 1

    cb = COLL_FN(coll)
    _keep.append(cb)
    _check("brd_dist_init_host", lib.brd_dist_init_host(rank, world, cb, None))


def finalize() -> None:
    _check("brd_dist_finalize", lib.brd_dist_finalize())
    _keep.clear()


# ---------------------------------------------------------------------------
# compute
# ---------------------------------------------------------------------------
def _local_ld(A_loc) -> int:
    """Leading dimension of a shard: its row stride (row-major, unit column
    stride), or 1 for an empty shard (n_loc == 0 on ranks without panels)."""
    if A_loc.dim() != 2:
        raise ValueError("A_loc must be a 2-D m x n_loc tensor")
    if A_loc.numel() == 0:
        return 1
    return _row_stride(A_loc)


def ge2band(A_loc, n: int, b: int, *, sync: bool = True):
    """Distributed dense -> band IN PLACE on this rank's shard ``A_loc``
    (torch CUDA tensor, m x n_loc, contiguous; n_loc may be 0).  Every rank
    of the communicator calls it.  Returns ``A_loc``."""
    m = A_loc.shape[0]
    sfx = _sfx(A_loc.dtype)
    _bind_stream(A_loc)
    ld = _local_ld(A_loc)
    ptr = A_loc.data_ptr() if A_loc.numel() else 0
    flags = BRD_DEVICE_PTR | (0 if sync else BRD_ASYNC)
    fn = f"brd_ge2band_dist_{sfx}"
    _check(fn, getattr(lib, fn)(ctypes.c_void_p(ptr), m, int(n), ld, int(b), flags))
    return A_loc


def gather_band(A_loc, n: int, b: int, root: int = 0, *, out=None, sync: bool = True):
    """Assemble the band (diagonals 0..b, zeros elsewhere) of the distributed
    stage-1 result on rank ``root`` as a dense m x n CUDA tensor; returns it on
    the root (``out`` if given) and ``None`` elsewhere."""
    import torch
    import torch.distributed as dist
    m = A_loc.shape[0]
    sfx = _sfx(A_loc.dtype)
    _bind_stream(A_loc)
    me = dist.get_rank()
    B: Optional[torch.Tensor] = None
    ldb = int(n)
    if me == root:
        B = out if out is not None else torch.empty((m, n), dtype=A_loc.dtype, device=A_loc.device)
        if tuple(B.shape) != (m, n) or B.dtype != A_loc.dtype:
            raise ValueError(f"out must be a {m} x {n} tensor of {A_loc.dtype}")
        ldb = _row_stride(B)
    ld = _local_ld(A_loc)
    ptr = A_loc.data_ptr() if A_loc.numel() else 0
    flags = BRD_DEVICE_PTR | (0 if sync else BRD_ASYNC)
    fn = f"brd_dist_gather_band_{sfx}"
    _check(fn, getattr(lib, fn)(ctypes.c_void_p(ptr), m, int(n), ld, int(b),
                                ctypes.c_void_p(B.data_ptr() if B is not None else 0), ldb, int(root), flags))
    return B

"""Python host side of the MI355X two-stage bidiagonal reduction.

Mirrors the reference's operator interface for the hot path:

* :func:`brd_p1` / :func:`cuda_brd_p1` -- dense -> band, like
  ``csc586::gpu::cuda_brd_p1(Matrix<float>& A, size_t b)`` (reference
  svd_cuda_2.cu:1117) and ``csc586::parallel::brd_p1<T>`` (svd_parallel.h:411):
  takes an N x N matrix and the band width b, returns the band matrix.
* :func:`brd_p2` -- band -> bidiagonal with the reference's window geometry,
  like ``csc586::parallel::brd_p2<T>`` (svd_parallel.h:640): returns the
  matrix after the sweeps plus the ``Bidiagonal{d, e}`` vectors.

Every call goes through the C ABI of ``lib/libbrd_hip.so`` (include/brd.h).
numpy arrays take the host-pointer path (the library stages them through
HBM); torch CUDA tensors are reduced in place on the device, on torch's
current stream.  There is no CPU fallback: if the HIP library is missing the
import of this module fails.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# BRD_LIB: another build of the same library (developer A/B runs)
LIB_PATH = os.environ.get("BRD_LIB") or os.path.join(_HERE, "lib", "libbrd_hip.so")

BRD_DEVICE_PTR = 0x1
BRD_ASYNC = 0x2
BRD_COMPAT = 0x0
BRD_EXACT_ORDER = 0x4
BRD_NO_EXTRACT = 0x8
BRD_SIGMA = 0x10

EXPORTED = (
    "brd_ge2band_f64", "brd_ge2band_f32", "brd_band2bd_f64", "brd_band2bd_f32",
    "brd_set_stream", "brd_use_own_stream", "brd_set_overlap", "brd_check_errors", "brd_release_stream", "brd_profile_enable", "brd_profile_reset", "brd_profile_query",
    "brd_dist_unique_id", "brd_dist_init", "brd_dist_init_host", "brd_dist_finalize", "brd_dist_local_cols",
    "brd_ge2band_dist_f64", "brd_ge2band_dist_f32", "brd_dist_gather_band_f64", "brd_dist_gather_band_f32",
    "brd_bdsvd_f64", "brd_bdsvd_f32", "brd_bdsvd_dev_f64", "brd_bdsvd_dev_f32", "brd_last_error", "brd_version",
)

# brd_coll_fn (include/brd.h): int (*)(int op, const void *send, void *recv,
#                                     unsigned long count, int dtype, int root, void *user)
COLL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p)


class BrdError(RuntimeError):
    """Raised when a libbrd_hip entry point returns a negative brd_status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C svdsolver_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    # torch bundles its own HIP runtime (torch/lib/libamdhip64.so, SONAME
    # libamdhip64.so.7).  Loaded after libbrd_hip.so (which needs
    # /opt/rocm's libamdhip64.so.7), torch would bring a second runtime that
    # does not know the library's device pointers and vice versa; loading
    # torch first lets the library bind to the runtime already in the process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, ci, cu = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint
    for t in ("f64", "f32"):
        f = getattr(L, f"brd_ge2band_{t}")
        f.argtypes = [vp, ci, ci, ci, ci, ci, cu]
        f.restype = ci
        g = getattr(L, f"brd_band2bd_{t}")
        g.argtypes = [vp, ci, ci, ci, vp, vp, cu]
        g.restype = ci
        h = getattr(L, f"brd_bdsvd_{t}")
        h.argtypes = [vp, vp, ci, vp]
        h.restype = ci
        hd = getattr(L, f"brd_bdsvd_dev_{t}")
        hd.argtypes = [vp, vp, ci, vp, cu]
        hd.restype = ci
    L.brd_set_stream.argtypes = [vp]
    L.brd_set_stream.restype = ci
    L.brd_use_own_stream.argtypes = []
    L.brd_use_own_stream.restype = ci
    L.brd_set_overlap.argtypes = [ci]
    L.brd_set_overlap.restype = ci
    L.brd_check_errors.argtypes = []
    L.brd_check_errors.restype = ci
    L.brd_release_stream.argtypes = [ctypes.c_void_p]
    L.brd_release_stream.restype = ci
    L.brd_profile_enable.argtypes = [ci]
    L.brd_profile_enable.restype = ci
    L.brd_profile_reset.argtypes = []
    L.brd_profile_reset.restype = ci
    L.brd_profile_query.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_double)]
    L.brd_profile_query.restype = ci
    L.brd_dist_unique_id.argtypes = [vp, ci]
    L.brd_dist_unique_id.restype = ci
    L.brd_dist_init.argtypes = [ci, ci, vp, ci]
    L.brd_dist_init.restype = ci
    L.brd_dist_init_host.argtypes = [ci, ci, COLL_FN, vp]
    L.brd_dist_init_host.restype = ci
    L.brd_dist_finalize.argtypes = []
    L.brd_dist_finalize.restype = ci
    L.brd_dist_local_cols.argtypes = [ci, ci, ci, ci]
    L.brd_dist_local_cols.restype = ci
    for t in ("f64", "f32"):
        f = getattr(L, f"brd_ge2band_dist_{t}")
        f.argtypes = [vp, ci, ci, ci, ci, cu]
        f.restype = ci
        g = getattr(L, f"brd_dist_gather_band_{t}")
        g.argtypes = [vp, ci, ci, ci, ci, vp, ci, ci, cu]
        g.restype = ci
    L.brd_last_error.argtypes = []
    L.brd_last_error.restype = ctypes.c_char_p
    L.brd_version.argtypes = []
    L.brd_version.restype = ci
    return L


lib = _load()


def _check(fn: str, rc: int) -> None:
    if rc != 0:
        raise BrdError(fn, rc, lib.brd_last_error().decode(errors="replace"))


def _sfx(dtype) -> str:
    s = str(dtype)
    if s in ("float64", "torch.float64"):
        return "f64"
    if s in ("float32", "torch.float32"):
        return "f32"
    raise TypeError(f"unsupported dtype {dtype} (float32 / float64 only)")


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def _bind_stream(x) -> None:
    import torch
    lib.brd_set_stream(ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))


def _row_stride(A) -> int:
    """Leading dimension of a row-major CUDA tensor: contiguous rows
    (stride(1) == 1) at any row stride >= n (lda, as in the C ABI)."""
    m, n = A.shape
    if A.stride(1) != 1 or A.stride(0) < n:
        raise ValueError("A must be row-major with unit column stride and row stride >= n")
    return int(A.stride(0))


# ---------------------------------------------------------------------------
# stage 1
# ---------------------------------------------------------------------------
def ge2band(A, b: int, *, sync: bool = True):
    """Dense -> band (bandwidth ``b``) IN PLACE.  ``A`` is a C-contiguous
    float32/float64 numpy array (host path) or torch CUDA tensor (device
    path, torch's current stream).  Returns ``A``."""
    m, n = A.shape
    sfx = _sfx(A.dtype)
    fn = f"brd_ge2band_{sfx}"
    if _is_torch_cuda(A):
        lda = _row_stride(A)
        _bind_stream(A)
        flags = BRD_DEVICE_PTR | (0 if sync else BRD_ASYNC)
        _check(fn, getattr(lib, fn)(ctypes.c_void_p(A.data_ptr()), m, n, lda, int(b), 1, flags))
    else:
        if not (isinstance(A, np.ndarray) and A.flags.c_contiguous):
            raise TypeError("host path needs a C-contiguous numpy array")
        _check(fn, getattr(lib, fn)(ctypes.c_void_p(A.ctypes.data), m, n, n, int(b), 1, 0))
    return A


def brd_p1(A, b: int):
    """Reference-compatible dense -> band: returns the band matrix (a copy for
    numpy input, like ``csc586::parallel::brd_p1`` returning ``Matrix``)."""
    if _is_torch_cuda(A):
        return ge2band(A.contiguous().clone(), b)
    return ge2band(np.array(A, copy=True, order="C"), b)


cuda_brd_p1 = brd_p1   # name of the reference GPU entry point (svd_cuda_2.cu:1117)


# ---------------------------------------------------------------------------
# stage 2
# ---------------------------------------------------------------------------
def band2bd(A, b: int, *, exact_order: bool = False, sigma: bool = False, sync: bool = True,
            extract: bool = True):
    """Band -> bidiagonal IN PLACE with the reference's window geometry, or
    (``sigma``) the sigma-preserving one: the bidiagonal then has the band's
    singular values (BRD_SIGMA, include/brd.h).
    Returns (d, e) (None, None when ``extract`` is False)."""
    m, n = A.shape
    assert m == n, "stage 2 takes a square band matrix"
    sfx = _sfx(A.dtype)
    fn = f"brd_band2bd_{sfx}"
    flags = ((BRD_EXACT_ORDER if exact_order else 0) | (BRD_SIGMA if sigma else 0)
             | (0 if extract else BRD_NO_EXTRACT))
    if _is_torch_cuda(A):
        import torch
        _bind_stream(A)
        d = torch.empty(n, dtype=A.dtype, device=A.device) if extract else None
        e = torch.empty(max(n - 1, 1), dtype=A.dtype, device=A.device) if extract else None
        flags |= BRD_DEVICE_PTR | (0 if sync else BRD_ASYNC)
        _check(fn, getattr(lib, fn)(ctypes.c_void_p(A.data_ptr()), n, _row_stride(A), int(b),
                                    ctypes.c_void_p(d.data_ptr() if extract else 0),
                                    ctypes.c_void_p(e.data_ptr() if extract else 0), flags))
        return (d, e[: n - 1]) if extract else (None, None)
    if not (isinstance(A, np.ndarray) and A.flags.c_contiguous):
        raise TypeError("host path needs a C-contiguous numpy array")
    d = np.zeros(n, dtype=A.dtype)
    e = np.zeros(max(n - 1, 1), dtype=A.dtype)
    _check(fn, getattr(lib, fn)(ctypes.c_void_p(A.ctypes.data), n, n, int(b),
                                ctypes.c_void_p(d.ctypes.data), ctypes.c_void_p(e.ctypes.data), flags))
    return (d, e[: n - 1]) if extract else (None, None)


def brd_p2(A, b: int, *, exact_order: bool = False, sigma: bool = False) -> Tuple[object, object, object]:
    """Reference-compatible band -> bidiagonal: returns (A_after, d, e), where
    A_after is what the reference writes to bidiagonal_*.bin (``sigma``: the
    sigma-preserving variant, not in the reference)."""
    B = A.contiguous().clone() if _is_torch_cuda(A) else np.array(A, copy=True, order="C")
    d, e = band2bd(B, b, exact_order=exact_order, sigma=sigma)
    return B, d, e


# ---------------------------------------------------------------------------
# bidiagonal -> singular values (host), and the whole pipeline
# ---------------------------------------------------------------------------
def bdsvd(d, e):
    """Singular values (descending) of the upper bidiagonal (d, e) via the
    library's host Golub-Kahan QR (brd_bdsvd_*; replaces the reference's
    serial::qrd, svd_serial.h:368).  d, e: numpy arrays or torch tensors."""
    if _is_torch_cuda(d):
        d, e = d.cpu().numpy(), e.cpu().numpy()
    d = np.ascontiguousarray(d)
    e = np.ascontiguousarray(e, dtype=d.dtype)
    n = d.shape[0]
    if e.shape[0] != max(n - 1, 0):
        raise ValueError("e must have n - 1 entries")
    sfx = _sfx(d.dtype)
    sv = np.empty(n, dtype=d.dtype)
    ep = e if n > 1 else np.zeros(1, dtype=d.dtype)
    fn = f"brd_bdsvd_{sfx}"
    _check(fn, getattr(lib, fn)(ctypes.c_void_p(d.ctypes.data), ctypes.c_void_p(ep.ctypes.data), n,
                                ctypes.c_void_p(sv.ctypes.data)))
    return sv


def bdsvd_gpu(d, e, *, sync: bool = True):
    """Singular values (descending) of the upper bidiagonal (d, e) on the GPU:
    multisection on the Golub-Kahan tridiagonal, every value bracketed on its
    own (brd_bdsvd_dev_*; the host twin is :func:`bdsvd`).  d, e: torch CUDA
    tensors of one dtype (e has n - 1 entries); returns a CUDA tensor."""
    import torch
    if not (_is_torch_cuda(d) and (_is_torch_cuda(e) or d.shape[0] == 1)):
        raise ValueError("bdsvd_gpu takes torch CUDA tensors (use bdsvd for host arrays)")
    d = d.contiguous()
    n = d.shape[0]
    if e.shape[0] != max(n - 1, 0):
        raise ValueError("e must have n - 1 entries")
    e = e.to(d.dtype).contiguous()
    sfx = _sfx(d.dtype)
    sv = torch.empty_like(d)
    _bind_stream(d)
    fn = f"brd_bdsvd_dev_{sfx}"
    _check(fn, getattr(lib, fn)(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(e.data_ptr() if n > 1 else 0), n,
                                ctypes.c_void_p(sv.data_ptr()), 0 if sync else BRD_ASYNC))
    return sv


def singular_values_gpu(A, b: int = 32):
    """Singular values of the square torch CUDA matrix A, every step on the GPU:
    stage 1, stage 2 with the sigma-preserving geometry, :func:`bdsvd_gpu`.
    A is not modified; returns a CUDA tensor (descending)."""
    M = A.clone()
    ge2band(M, b)
    d, e = band2bd(M, b, sigma=True)
    return bdsvd_gpu(d, e)


def singular_values(A, b: int = 32):
    """Singular values of the square matrix A: stage 1 (dense -> band, GPU),
    stage 2 with the sigma-preserving geometry (GPU), then bdsvd (host).
    A is not modified."""
    B = brd_p1(A, b)
    _, d, e = brd_p2(B, b, sigma=True)
    return bdsvd(d, e)


# ---------------------------------------------------------------------------
# stream of reductions: stage 2 of one matrix beside stage 1 of the next
# ---------------------------------------------------------------------------
def set_overlap(s2_cus: int) -> None:
    """brd_set_overlap (include/brd.h): run stage-2 sweeps on ``s2_cus``
    workgroups and size stage-1 launches for the remaining CUs, so that a
    band2bd on one stream and a ge2band on another share the chip; 0 restores
    the whole-chip defaults."""
    _check("brd_set_overlap", lib.brd_set_overlap(int(s2_cus)))


def overlap_cus(n: int) -> int:
    """CUs reserved for stage 2 when it overlaps stage 1.  Measured on MI355X
    (profiles/README.md, pipelined bench at n = 8192): 32 workgroups keep the
    sweep chain within 1 % of its whole-chip time and leave 224 CUs (28 per
    XCD) to stage 1 (93.7 ms beside the sweep, 88 ms alone); 64 gave 101.7 ms,
    and 40-56 or 72-128 were slower still (fp32: 16 and 24 slower than 32 too;
    the good values are multiples of 32, see profiles/README.md).  Stage 1
    dominates at larger n, so the reservation stays at 32."""
    return 32 if n >= 1024 else 16


def reduce_many(mats, b: int, *, sigma: bool = False, s2_cus: Optional[int] = None, sync: bool = True,
                lanes: int = 1, s2_lanes: Optional[int] = None):
    """Two-stage reduction of a sequence of square CUDA tensors, each in place,
    pipelined over pairs of HIP streams ("lanes"): on a lane, stage 2 of
    matrix i (its own stream, ``s2_cus`` workgroups) runs beside stage 1 of the
    lane's next matrix (the other stream, sized for the remaining CUs); matrix
    i goes to lane i mod ``lanes``.  Returns [(d, e)] per matrix (device
    tensors).  Each matrix sees exactly the calls of ge2band + band2bd; only
    their overlap differs.  The library's overlap setting is restored on exit.
    More than one lane pays only with one hardware queue per stream: set
    GPU_MAX_HW_QUEUES >= lanes + s2_lanes + 4 (at most 32) before HIP
    initialises ("lanes").  ``s2_lanes``: stage-2 streams (matrix
    i's stage 2 on stream i mod s2_lanes; default one per lane): fewer than
    the lanes make a burst of finished stage 1s queue for the sweep instead of
    each taking ``s2_cus`` CUs at once (bench.py: 10 lanes, 5 stage-2 streams).
    """
    import torch
    if not mats:
        return []
    if lanes < 1:
        raise ValueError("lanes must be >= 1")
    dev = mats[0].device
    cus = overlap_cus(mats[0].shape[0]) if s2_cus is None else int(s2_cus)
    lanes = min(int(lanes), len(mats))
    s2l = lanes if s2_lanes is None else max(1, min(int(s2_lanes), len(mats)))
    # every lane's stage-2 kernel is a persistent grid of ``cus`` workgroups,
    # one per CU (its LDS ring takes the CU), whose bundles wait on each
    # other: with more workgroups in flight than the chip holds, a partly
    # resident grid stalls ("Overlap and lanes")
    dev_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    if s2l * cus > dev_cus:
        raise ValueError(f"stage-2 streams * s2_cus = {s2l} * {cus} exceeds the device's {dev_cus} CUs "
                         "(stage-2 grids must fit the chip together)")
    s_a = [torch.cuda.Stream(dev) for _ in range(lanes)]
    s_b = [torch.cuda.Stream(dev) for _ in range(s2l)]
    for s in s_a:
        s.wait_stream(torch.cuda.current_stream(dev))
    out = []
    set_overlap(cus)
    try:
        for i, A in enumerate(mats):
            sa, sb = s_a[i % lanes], s_b[i % s2l]
            with torch.cuda.stream(sa):
                ge2band(A, b, sync=False)
                done1 = torch.cuda.Event()
                done1.record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(done1)
                out.append(band2bd(A, b, sigma=sigma, sync=False))
    finally:
        set_overlap(0)
    for s in s_b:
        torch.cuda.current_stream(dev).wait_stream(s)
    if sync:
        torch.cuda.synchronize(dev)
        check_errors()
    return out


def release_stream(stream=None) -> None:
    """brd_release_stream (include/brd.h): drain ``stream`` (a torch CUDA
    stream; None: the library's current stream) and free the library's
    per-stream workspaces, staging buffer and error word; call before the
    stream is destroyed."""
    h = None if stream is None else ctypes.c_void_p(stream.cuda_stream)
    _check("brd_release_stream", lib.brd_release_stream(h))


def check_errors() -> None:
    """brd_check_errors (include/brd.h): drain the library's streams and raise
    :class:`BrdError` if an asynchronous stage-2 sweep hit its spin limit (its
    output is invalid) or a HIP error is pending."""
    _check("brd_check_errors", lib.brd_check_errors())


# ---------------------------------------------------------------------------
# profiling (per-kernel HIP-event timing inside the library)
# ---------------------------------------------------------------------------
def profile_enable(on: bool = True) -> None:
    _check("brd_profile_enable", lib.brd_profile_enable(1 if on else 0))


def profile_reset() -> None:
    _check("brd_profile_reset", lib.brd_profile_reset())


def profile_query(kernel: str) -> dict:
    n = ctypes.c_longlong()
    ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    _check("brd_profile_query", lib.brd_profile_query(kernel.encode(), ctypes.byref(n), ctypes.byref(ms),
                                                      ctypes.byref(fl), ctypes.byref(by)))
    return {"launches": n.value, "ms": ms.value, "flops": fl.value, "bytes": by.value}

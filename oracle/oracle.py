"""TEST INFRASTRUCTURE ONLY: ctypes front end of the CPU oracle.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module.  The product path (``svdsolver_amd``) never does.

The oracle (``brd_oracle_impl.h``) restates the reference's CPU tiled
algorithm -- ``csc586::parallel::brd_p1`` (svd_parallel.h:411-533) and
``csc586::parallel::brd_p2`` (svd_parallel.h:640-695) -- operation for
operation, so it reproduces the reference's fixtures bit for bit.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    """Compile liboracle.so with the oracle's Makefile (no fp contraction)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        for sfx in ("f32", "f64"):
            f = getattr(L, f"oracle_brd_p1_{sfx}")
            f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
            f.restype = ctypes.c_int
            g = getattr(L, f"oracle_brd_p2_{sfx}")
            g.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
            g.restype = ctypes.c_int
            g = getattr(L, f"oracle_brd_p2x_{sfx}")
            g.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
            g.restype = ctypes.c_int
        _lib = L
    return _lib


def _sfx(a: np.ndarray) -> str:
    if a.dtype == np.float32:
        return "f32"
    if a.dtype == np.float64:
        return "f64"
    raise TypeError(f"oracle supports float32/float64, got {a.dtype}")


def brd_p1(A: np.ndarray, t: int) -> np.ndarray:
    """Dense -> band, reference tiled algorithm (svd_parallel.h:411). Returns a copy."""
    A = np.ascontiguousarray(A).copy()
    n = A.shape[0]
    assert A.shape == (n, n)
    rc = getattr(lib(), f"oracle_brd_p1_{_sfx(A)}")(A.ctypes.data, n, n, int(t))
    if rc != 0:
        raise ValueError(f"oracle_brd_p1 failed rc={rc} (n={n}, t={t}: t must divide n)")
    return A


def brd_p2(A: np.ndarray, b: int, sigma: bool = False):
    """Band -> bidiagonal, reference windowed sweep (svd_parallel.h:640).

    Returns (A_out, d, e) where A_out is the full matrix after the sweeps
    (what the reference writes to bidiagonal_*.bin).  sigma=True: the
    sigma-preserving variant (one more window pair per sweep; not in the
    reference, see brd_oracle_impl.h)."""
    A = np.ascontiguousarray(A).copy()
    m, n = A.shape
    d = np.zeros(n, dtype=A.dtype)
    e = np.zeros(max(n - 1, 0), dtype=A.dtype)
    rc = getattr(lib(), f"oracle_brd_p2x_{_sfx(A)}")(A.ctypes.data, m, n, n, int(b),
                                                      d.ctypes.data, e.ctypes.data, int(bool(sigma)))
    if rc != 0:
        raise ValueError(f"oracle_brd_p2 failed rc={rc}")
    return A, d, e

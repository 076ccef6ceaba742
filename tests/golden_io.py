"""Loaders for the committed golden vectors (tests/golden/, see make_golden.py)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TYPES = {"float": np.float32, "double": np.float64}


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def ref_bin(name: str, n: int, T: str) -> np.ndarray:
    return np.fromfile(os.path.join(GOLDEN, "ref_data", name), dtype=TYPES[T]).reshape(n, n)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def npz(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def diags(a: np.ndarray, lo: int, hi: int) -> np.ndarray:
    n = a.shape[0]
    out = np.zeros((hi - lo + 1, n), dtype=a.dtype)
    for r, off in enumerate(range(lo, hi + 1)):
        dg = np.diagonal(a, off)
        out[r, : dg.size] = dg
    return out


def input1024(T: str) -> np.ndarray:
    from splitmix import uniform_matrix
    return uniform_matrix(1024, seed=1024, lo=1.0, hi=5.0, dtype=np.float64).astype(TYPES[T])


def band_abs_err(a: np.ndarray, ref: np.ndarray, b: int):
    """Normwise and max-abs error of |a| vs |ref| over the upper band
    (diagonals 0..b), the region the reference's own metric compares
    (matrix_gpu.h:438-453; sign-insensitive)."""
    n = a.shape[0]
    i, j = np.indices((n, n))
    m = (j >= i) & (j - i <= b)
    da = np.abs(a[m]).astype(np.float64) - np.abs(ref[m]).astype(np.float64)
    nr = np.linalg.norm(ref[m].astype(np.float64))
    return float(np.linalg.norm(da) / nr), float(np.max(np.abs(da)))


def ref_mse(a: np.ndarray, ref: np.ndarray, band_size: int) -> float:
    """The reference's Matrix::mse(B, band_size) (matrix_gpu.h:438-453):
    sum over i, j in [i, i+band_size) of ||a_ij| - |b_ij|| / (band_size * n)."""
    n = a.shape[0]
    i, j = np.indices((n, n))
    m = (j >= i) & (j < i + band_size)
    return float(np.sum(np.abs(np.abs(a[m].astype(np.float64)) - np.abs(ref[m].astype(np.float64)))) / (band_size * n))

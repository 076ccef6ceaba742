"""Deterministic input generator for golden vectors and benchmarks.

splitmix64 (Steele, Lea, Flood 2014) -> 53-bit uniform in [0,1) -> [lo, hi).
Pure numpy (uint64 wrap-around arithmetic), so the same matrices can be
regenerated on the GPU box without shipping them.  The reference fixtures use
values in [1,5); its benchmarks use [0,5) (svd_cuda_2.cu:1361).
"""
import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int) -> np.ndarray:
    idx = np.arange(1, count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform_matrix(n: int, seed: int, lo: float = 1.0, hi: float = 5.0,
                   dtype=np.float64) -> np.ndarray:
    u = (splitmix64(seed, n * n) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return (lo + (hi - lo) * u).reshape(n, n).astype(dtype)

"""svdsolver_amd: MI355X-native two-stage bidiagonal reduction (dense -> band
-> bidiagonal), a drop-in for the GPU path of scrose/SVDSolver.

The compute path is libbrd_hip.so (hand-written gfx950 HIP kernels behind the
C ABI in include/brd.h); this package is its Python host side.
"""
from .brd import (BRD_DEVICE_PTR, BRD_EXACT_ORDER, BRD_NO_EXTRACT, BRD_SIGMA, BrdError, LIB_PATH,  # noqa: F401
                  band2bd, bdsvd, bdsvd_gpu, brd_p1, brd_p2, check_errors, cuda_brd_p1, ge2band, lib, profile_enable,
                  profile_query, profile_reset, reduce_many, release_stream, set_overlap, overlap_cus, singular_values,
                  singular_values_gpu)

__all__ = ["ge2band", "band2bd", "reduce_many", "brd_p1", "brd_p2", "cuda_brd_p1", "bdsvd", "bdsvd_gpu", "singular_values",
           "singular_values_gpu", "BrdError"]

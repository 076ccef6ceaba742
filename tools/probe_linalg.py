"""Timing probe (developer tool): how long rocSOLVER's fp64 eigvalsh(A^T A) and
svdvals take at the bench sizes -- sizing the reference checks of
tests/test_gpu_large.py."""
import time

import torch

for n in (8192, 16384):
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.rand(n, n, dtype=torch.float64, device="cuda", generator=g) * 5
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    G = A.T @ A
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    lam = torch.linalg.eigvalsh(G)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n}: gram {t1 - t0:.2f} s, eigvalsh {t2 - t1:.2f} s, lam_max {float(lam[-1]):.6e}", flush=True)
    del G, lam
    if n == 8192:
        t0 = time.perf_counter()
        s = torch.linalg.svdvals(A)
        torch.cuda.synchronize()
        print(f"n={n}: svdvals {time.perf_counter() - t0:.2f} s, smax {float(s[0]):.6e}", flush=True)
    del A
    torch.cuda.empty_cache()

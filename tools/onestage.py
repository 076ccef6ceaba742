"""One-stage bidiagonalisation on the GPU as a comparison baseline (SURVEY.md
8(f) rank 4; the reference's CPU `base`/`singlecore` models): brd_ge2band with
band width 1 IS the classic alternating Householder QR/LQ reduction straight
to bidiagonal form (BLAS-2: every column/row reflector re-reads the whole
trailing matrix).  Prints GFLOP/s (8/3 N^3) against the two-stage path.

usage: python tools/onestage.py [N] [dtype f64|f32]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dt = torch.float64 if (len(sys.argv) < 3 or sys.argv[2] == "f64") else torch.float32
g = torch.Generator(device="cuda").manual_seed(3)
A0 = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
flops = 8.0 / 3.0 * n ** 3


def timed(fn, reps=2):
    best = 1e30
    for _ in range(reps + 1):
        A = A0.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(A)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


t1 = timed(lambda A: S.ge2band(A, 1))
t2 = timed(lambda A: (S.ge2band(A, 32), S.band2bd(A, 32, extract=False)))
print(f"N={n} {sys.argv[2] if len(sys.argv) > 2 else 'f64'}: one-stage (band 1) {t1 * 1e3:.1f} ms "
      f"{flops / t1 / 1e9:.0f} GFLOP/s | two-stage (band 32) {t2 * 1e3:.1f} ms {flops / t2 / 1e9:.0f} GFLOP/s "
      f"| speedup {t1 / t2:.2f}x")

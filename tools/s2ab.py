"""Stage-2 A/B (developer tool): k_sweeps (default) vs k_band2bd_bundle
(BRD_S2_LEGACY=1) on the same bands: time (median of runs) and the |d|, |e|
deviation between them and against the exact-order sweep's rounding envelope.
usage: python tools/s2ab.py N[,N...] [f32] [runs]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

ns = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2048,8192").split(",")]
dt = torch.float32 if (len(sys.argv) > 2 and sys.argv[2] == "f32") else torch.float64
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
b = 32


def bd_err(d, e, d0, e0):
    got = torch.cat([d.abs(), e.abs()]).double()
    ref = torch.cat([d0.abs(), e0.abs()]).double()
    return float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref))


def sweep(band, legacy, exact=False):
    os.environ["BRD_S2_LEGACY"] = "1" if legacy else "0"
    ts, out = [], None
    for _ in range(1 if exact else runs):
        W = band.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d, e = S.band2bd(W, b, exact_order=exact)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        S.check_errors()
        if out is not None:
            assert torch.equal(out[0], d) and torch.equal(out[1], e), "not run-to-run reproducible"
        out = (d.clone(), e.clone())
    ts.sort()
    return out, ts[len(ts) // 2]


for n in ns:
    g = torch.Generator(device="cuda").manual_seed(n)
    A = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
    S.ge2band(A, b)
    (d1, e1), t1 = sweep(A, False)
    (d0, e0), t0 = sweep(A, True)
    (dx, ex), _ = sweep(A, False, exact=True)
    eps = float(torch.finfo(dt).eps)
    p = A * (1 + eps * torch.randn(A.shape, dtype=dt, device="cuda", generator=g))
    (dp, ep), _ = sweep(p, False, exact=True)
    env = bd_err(dp, ep, dx, ex)
    print(f"n={n} {dt}: k_sweeps {t1:.2f} ms, legacy {t0:.2f} ms | dev new-vs-exact {bd_err(d1, e1, dx, ex):.2e} "
          f"legacy-vs-exact {bd_err(d0, e0, dx, ex):.2e} envelope {env:.2e} finite {bool(torch.isfinite(d1).all())}",
          flush=True)

"""GPU bidiagonal singular values: timing and agreement with the host QR
(developer tool).  usage: python tools/bd_time.py [n] [tag]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
tag = sys.argv[2] if len(sys.argv) > 2 else "run"
rng = np.random.default_rng(17)
d, e = rng.uniform(-2, 2, n), rng.uniform(-2, 2, n - 1)
td, te = torch.from_numpy(d).cuda(), torch.from_numpy(e).cuda()
S.bdsvd_gpu(td, te)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    got = S.bdsvd_gpu(td, te)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
ref = S.bdsvd(d, e)
err = float(np.max(np.abs(got.cpu().numpy() - ref)) / ref[0])
print(f"{tag}: n={n} GPU median {np.median(ts):.2f} ms, max |err| / sigma_max {err:.2e}")

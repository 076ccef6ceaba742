"""Stage-2 timing under the current environment (developer tool): band2bd on
an N x N band (b = 32, fp64) resident on the GPU, median of a few runs, plus
an agreement check against the first variant's output saved in /tmp."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
tag = sys.argv[2] if len(sys.argv) > 2 else "run"
dt = torch.float32 if (len(sys.argv) > 3 and sys.argv[3] == "f32") else torch.float64
b = 32
g = torch.Generator(device="cuda").manual_seed(5)
A0 = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 4 + 1
i = torch.arange(n, device="cuda")
mask = (i[None, :] >= i[:, None]) & (i[None, :] - i[:, None] <= b)
A0 = A0 * mask
ts = []
for it in range(4):
    A = A0.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d, e = S.band2bd(A, b)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
ref = "/tmp/s2time_ref.npy"
dd = d.cpu().numpy()
if not os.path.exists(ref):
    np.save(ref, dd)
    dev = 0.0
else:
    r = np.load(ref)
    dev = float(np.linalg.norm(np.abs(dd) - np.abs(r)) / np.linalg.norm(r))
print(f"{tag}: stage2 n={n} {dt} median {np.median(ts):.2f} ms (runs {', '.join(f'{t:.1f}' for t in ts)}) |d| dev vs first {dev:.2e}")

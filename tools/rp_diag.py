"""Developer diagnostic: a few stage-1 reductions at N = 8192 fp64 under the
library given by BRD_LIB (e.g. a diagnostic build whose results are wrong by
construction), errors ignored: for rocprofv3 kernel statistics only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g = torch.Generator(device="cuda").manual_seed(5)
A0 = torch.rand(n, n, dtype=torch.float64, device="cuda", generator=g) * 5
for _ in range(3):
    A = A0.clone()
    try:
        S.ge2band(A, 32)
    except Exception as e:   # noqa: BLE001 -- diagnostic builds may trip the error word
        print("ignored:", str(e)[:80])
torch.cuda.synchronize()
print("done")

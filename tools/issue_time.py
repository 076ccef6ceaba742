"""Host time of the library's launch calls (developer tool): how long each
async ge2band / band2bd call takes to RETURN on an idle GPU versus the GPU
time, i.e. whether issuing blocks on the device (launch-queue capacity).
usage: python tools/issue_time.py [n=8192] [calls=4]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
A0 = torch.rand(n, n, dtype=torch.float64, device="cuda") * 5
M = A0.clone()
S.ge2band(M, 32)
S.band2bd(M, 32, extract=False)
torch.cuda.synchronize()
for what in ("ge2band", "band2bd", "ge2band on 2 streams"):
    mats = [A0.clone() for _ in range(k)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ts = []
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    for i, Mi in enumerate(mats):
        t = time.perf_counter()
        if what == "ge2band":
            S.ge2band(Mi, 32, sync=False)
        elif what == "band2bd":
            S.band2bd(Mi, 32, sync=False, extract=False)
        else:
            with torch.cuda.stream(streams[i % 2]):
                S.ge2band(Mi, 32, sync=False)
        ts.append(1e3 * (time.perf_counter() - t))
    t_issue = 1e3 * (time.perf_counter() - t0)
    torch.cuda.synchronize()
    t_all = 1e3 * (time.perf_counter() - t0)
    print(f"{what:22s} n={n}: per-call host ms {[round(x, 1) for x in ts]}, issue {t_issue:.1f} ms, done {t_all:.1f} ms")
    S.check_errors()

"""Run-to-run reproducibility probe of stage 1 (developer tool): for each
environment variant (';'-separated 'K=V K2=V2'), run ge2band on the same
matrix 3 times and report whether the bands agree bitwise and, if not, the
first differing column.  usage: python tools/s1_repro.py N 'VARS;VARS2'"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import svdsolver_amd as S

n = int(sys.argv[1])
dt = torch.float32 if os.environ.get("DT") == "f32" else torch.float64
variants = sys.argv[2].split(";") if len(sys.argv) > 2 else ["BASE=1"]
g = torch.Generator(device="cuda"); g.manual_seed(77)
A = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
for v in variants:
    saved = {}
    for kv in v.split():
        k, val = kv.split("=")
        saved[k] = os.environ.get(k); os.environ[k] = val
    outs = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        M = A.clone(); S.ge2band(M, 32); torch.cuda.synchronize(); outs.append(M)
    res = []
    for r in outs[1:]:
        if torch.equal(outs[0], r):
            res.append("equal")
        else:
            dif = (outs[0] != r)
            cols = torch.nonzero(dif.any(dim=0)).flatten()
            rows = torch.nonzero(dif.any(dim=1)).flatten()
            mx = float((outs[0] - r).abs().max())
            res.append(f"DIFF cols {int(cols[0])}..{int(cols[-1])} rows {int(rows[0])}..{int(rows[-1])} n={int(dif.sum())} max {mx:.2e}")
    print(v, "|", "; ".join(res), flush=True)
    for k, val in saved.items():
        if val is None: os.environ.pop(k, None)
        else: os.environ[k] = val

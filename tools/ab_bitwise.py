"""Bitwise A/B of two builds of the library (developer tool): stage 1 and the
compat stage 2 of the same seeded N x N matrix through each library's C ABI.
usage: [BRD_AB_OVERLAP=CUS] python tools/ab_bitwise.py <libA.so> <libB.so> [n=2048] [f64|f32]"""
import ctypes
import os
import sys

import torch

libs = [ctypes.CDLL(p) for p in sys.argv[1:3]]
ov = int(os.environ.get("BRD_AB_OVERLAP", "0"))   # > 0: stage 1 sized beside a stage-2 reservation (stream form)
for L in libs:
    assert L.brd_set_overlap(ov) == 0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
dt = torch.float32 if (len(sys.argv) > 4 and sys.argv[4] == "f32") else torch.float64
sfx = "f32" if dt == torch.float32 else "f64"
g = torch.Generator(device="cuda").manual_seed(n)
A0 = torch.rand(n, n, dtype=dt, device="cuda", generator=g) * 5
outs = []
for L in libs:
    A = A0.clone()
    d = torch.empty(n, dtype=dt, device="cuda")
    e = torch.empty(n - 1, dtype=dt, device="cuda")
    assert getattr(L, "brd_ge2band_" + sfx)(ctypes.c_void_p(A.data_ptr()), n, n, n, 32, 1, 1) == 0   # BRD_DEVICE_PTR
    band = A.clone()
    assert getattr(L, "brd_band2bd_" + sfx)(ctypes.c_void_p(A.data_ptr()), n, n, 32, ctypes.c_void_p(d.data_ptr()),
                                            ctypes.c_void_p(e.data_ptr()), 1) == 0
    assert L.brd_check_errors() == 0
    torch.cuda.synchronize()
    outs.append((band, A, d, e))
names = ["band", "bidiagonal matrix", "d", "e"]
for k in range(4):
    eq = torch.equal(outs[0][k], outs[1][k])
    dev = float((outs[0][k].double() - outs[1][k].double()).abs().max())
    print(f"n={n} {sfx} {names[k]}: bitwise equal {eq} (max |diff| {dev:.3e})")

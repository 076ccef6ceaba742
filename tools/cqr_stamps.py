"""Phase timing inside the panel-QR kernel k_cqr_v (developer tool): a
-DBRD_CQR_STAMPS build (bash tools/variant_lib.sh cqrst "-DBRD_CQR_STAMPS"
brd_blk_cqr.hip) records per-workgroup s_memrealtime stamps (100 MHz) of the
k_cqr_v launches whose panel height equals a target; one N x N fp64 ge2band
per target (the last matching launch of the call is reported).
usage: BRD_LIB=tools/ablib/cqrst.so python tools/cqr_stamps.py [n=8192] [panel ...]"""
import ctypes
import os
import sys

import torch

lib_path = os.environ.get("BRD_LIB")
assert lib_path and "cqrst" in lib_path, "BRD_LIB must name a -DBRD_CQR_STAMPS build"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import svdsolver_amd as S  # noqa: E402

L = ctypes.CDLL(lib_path)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
panels = [int(x) for x in sys.argv[2:]] or [8, 100, 200]
g = torch.Generator(device="cuda").manual_seed(n)
A0 = torch.rand(n, n, dtype=torch.float64, device="cuda", generator=g) * 5
A = A0.clone()
S.ge2band(A, 32)
torch.cuda.synchronize()
names = ["entry", "exponent", "gram sum", "chol/fast", "R2 solve", "store V", "zeros"]
for p in panels:
    M = n - 32 * p
    assert L.brd_debug_cqr_target(ctypes.c_long(M)) == 0
    A = A0.clone()
    S.ge2band(A, 32)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (64 * 12))()
    assert L.brd_debug_cqr_stamps(buf) == 0
    nwg = min(64, (M + 255) // 256)
    st = [[buf[w * 12 + q] for q in range(len(names))] for w in range(nwg)]
    st = [s for s in st if all(s)]
    if not st:
        print(f"panel {p}: M = {M}: no stamps")
        continue
    t0 = min(s[0] for s in st)
    print(f"panel {p}: M = {M}, k_cqr_v {len(st)} workgroups, first entry to last stamp "
          f"{(max(s[-1] for s in st) - t0) / 100:.2f} us, entry skew {(max(s[0] for s in st) - t0) / 100:.2f} us")
    for q in range(1, len(names)):
        d = sorted((s[q] - s[q - 1]) / 100 for s in st)
        print(f"    {names[q]:12s} median {d[len(d) // 2]:6.2f}  max {d[-1]:6.2f} us")

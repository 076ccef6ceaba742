"""Generate the committed golden vectors under tests/golden/.

Run in the development container (where /root/reference exists):
    python tests/golden/make_golden.py

What it writes
--------------
ref_data/test_{float,double}_{64,512}.bin, ref_data/{band,bidiagonal}_*_64_64.bin
    Copies of the reference's own fixture files (reference data/, raw
    row-major little-endian, no header).  The 512 outputs are large, so for
    them only their band diagonals and SHA-256 digests are kept:
ref512.npz
    band_{T}: diagonals -1..5 of band_{T}_512_512.bin (b=4)
    bidiagonal_{T}: diagonals -1..2 of bidiagonal_{T}_512_512.bin
gen1024.npz
    The reference ships no 1024 fixtures (its .MISSING_LARGE_BLOBS), so they
    are regenerated: input = splitmix.uniform_matrix(1024, seed=1024, 1, 5)
    (float32: the float64 matrix rounded), band = oracle brd_p1(A, b),
    bidiagonal = oracle brd_p2(band, b), for b = 4 (the reference `check`
    band) and b = 32 (the benchmark band), float64 and float32.  Stored as
    band diagonals plus SHA-256 digests of the full matrices.
manifest.json
    SHA-256 of every full fixture (signed bytes), and which generator
    produced it.  When oracle/_ref/libref.so (the reference's own headers
    compiled by oracle/Makefile) is present, every generated output is also
    produced by the reference build and must agree bit for bit.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import oracle  # noqa: E402  (test infrastructure)
from splitmix import uniform_matrix  # noqa: E402

REF_DATA = "/root/reference/data"
TYPES = {"float": np.float32, "double": np.float64}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def diags(a: np.ndarray, lo: int, hi: int) -> np.ndarray:
    n = a.shape[0]
    out = np.zeros((hi - lo + 1, n), dtype=a.dtype)
    for r, off in enumerate(range(lo, hi + 1)):
        dg = np.diagonal(a, off)
        out[r, : dg.size] = dg
    return out


def ref_lib():
    p = os.path.join(REPO, "oracle", "_ref", "libref.so")
    return ctypes.CDLL(p) if os.path.exists(p) else None


def main() -> None:
    os.makedirs(os.path.join(HERE, "ref_data"), exist_ok=True)
    manifest = {"ref_data": {}, "ref512": {}, "gen1024": {}}
    # --- reference fixtures ------------------------------------------------
    for T in TYPES:
        for N in (64, 512):
            name = f"test_{T}_{N}_{N}.bin"
            shutil.copyfile(os.path.join(REF_DATA, name), os.path.join(HERE, "ref_data", name))
        for kind in ("band", "bidiagonal"):
            name = f"{kind}_{T}_64_64.bin"
            shutil.copyfile(os.path.join(REF_DATA, name), os.path.join(HERE, "ref_data", name))
    for fn in sorted(os.listdir(REF_DATA)):
        if fn.endswith(".bin"):
            with open(os.path.join(REF_DATA, fn), "rb") as f:
                manifest["ref_data"][fn] = hashlib.sha256(f.read()).hexdigest()
    r512 = {}
    for T, dt in TYPES.items():
        band = np.fromfile(os.path.join(REF_DATA, f"band_{T}_512_512.bin"), dtype=dt).reshape(512, 512)
        bid = np.fromfile(os.path.join(REF_DATA, f"bidiagonal_{T}_512_512.bin"), dtype=dt).reshape(512, 512)
        r512[f"band_{T}"] = diags(band, -1, 5)
        r512[f"bidiagonal_{T}"] = diags(bid, -1, 2)
    np.savez(os.path.join(HERE, "ref512.npz"), **r512)
    manifest["ref512"] = {"band_diag_offsets": [-1, 5], "bidiagonal_diag_offsets": [-1, 2]}

    # --- regenerated 1024 --------------------------------------------------
    R = ref_lib()
    g = {}
    A64 = uniform_matrix(1024, seed=1024, lo=1.0, hi=5.0, dtype=np.float64)
    for T, dt in TYPES.items():
        A = A64.astype(dt)
        manifest["gen1024"][f"test_{T}"] = sha(A)
        for b in (4, 32):
            band = oracle.brd_p1(A, b)
            bid, d, e = oracle.brd_p2(band, b)
            key = f"{T}_b{b}"
            g[f"band_{key}"] = diags(band, -1, b + 1)
            g[f"bidiagonal_{key}"] = diags(bid, -1, 2)
            manifest["gen1024"][f"band_{key}"] = sha(band)
            manifest["gen1024"][f"bidiagonal_{key}"] = sha(bid)
            if R is not None:
                sfx = "f32" if dt == np.float32 else "f64"
                Rb = A.copy()
                getattr(R, f"ref_brd_p1_{sfx}")(Rb.ctypes.data_as(ctypes.c_void_p), 1024, b)
                Rc = Rb.copy()
                getattr(R, f"ref_brd_p2_{sfx}")(Rc.ctypes.data_as(ctypes.c_void_p), 1024, b)
                ok = np.array_equal(Rb, band) and np.array_equal(Rc, bid)
                manifest["gen1024"][f"reference_build_agrees_{key}"] = bool(ok)
                print(key, "reference build agrees bit-for-bit:", ok, flush=True)
                assert ok
            print("generated", key, flush=True)
    np.savez(os.path.join(HERE, "gen1024.npz"), **g)
    manifest["gen1024"]["input"] = "splitmix.uniform_matrix(1024, seed=1024, lo=1, hi=5); float32 = rounded float64"
    manifest["gen1024"]["band_diag_offsets"] = "[-1, b+1]"
    manifest["gen1024"]["bidiagonal_diag_offsets"] = [-1, 2]
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

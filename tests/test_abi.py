"""CPU-side checks of the C-ABI boundary: the library builds for gfx950,
loads, exports every symbol include/brd.h declares, and rejects bad
arguments before touching a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "brd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(brd_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("brd_ge2band_f64", "brd_ge2band_f32", "brd_band2bd_f64", "brd_band2bd_f32",
              "brd_last_error", "brd_set_stream", "brd_profile_query", "brd_dist_init"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import svdsolver_amd
    lib = ctypes.CDLL(svdsolver_amd.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), f"{s} declared in include/brd.h but not exported"
    assert set(declared_symbols()) <= set(svdsolver_amd.brd.EXPORTED)


def test_library_is_gfx950():
    import svdsolver_amd
    data = open(svdsolver_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("bad", [
    dict(m=4, n=8, b=4),      # m < n
    dict(m=8, n=8, b=0),      # b < 1
    dict(m=8, n=8, b=33),     # b > 32
])
def test_ge2band_rejects_bad_arguments(bad):
    import svdsolver_amd as S
    A = np.zeros((bad["m"], bad["n"]))
    rc = S.lib.brd_ge2band_f64(A.ctypes.data, bad["m"], bad["n"], bad["n"], bad["b"], 1, 0)
    assert rc == -1
    assert S.lib.brd_last_error()


def test_null_pointer_rejected():
    import svdsolver_amd as S
    assert S.lib.brd_ge2band_f32(None, 8, 8, 8, 4, 1, 0) == -1
    assert b"NULL" in S.lib.brd_last_error()
    assert S.lib.brd_band2bd_f64(None, 8, 8, 4, None, None, 0) == -1


def test_python_mirror_raises_brd_error():
    import svdsolver_amd as S
    with pytest.raises(S.BrdError):
        S.ge2band(np.zeros((8, 8)), 40)
    with pytest.raises(TypeError):
        S.ge2band(np.zeros((8, 8), dtype=np.int32), 4)

"""CPU test of the C++ boundary type include/brd_matrix.hpp (the stand-in for
the reference's csc586::gpu::Matrix<T>, matrix_gpu.h:79-535): tests/cpp/
test_matrix.cpp is compiled with g++ and run; it exercises every member the
reference defines (element access, +=/-=/*=, transpose, mm, flatten/reshape,
slice/copy/concat/fill/tiles, mse, read/write, Slice, Reflection)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_brd_matrix_hpp(tmp_path):
    exe = tmp_path / "test_matrix"
    src = os.path.join(REPO, "tests", "cpp", "test_matrix.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    src, "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ALL OK" in out.stdout

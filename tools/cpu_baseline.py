"""CPU baseline per BASELINE.md section 2 (developer tool; run on the GPU box's host,
nothing else running): the reference's tiled two-stage algorithm
(parallel::brd_p1 + brd_p2, svd_parallel.h:411/:640) compiled from its own
sources (oracle/_ref, README.md:32 flags minus -march=native), b = 32,
seeded uniform [0,5) inputs, OpenMP threads = the job's CPU share
(OMP_NUM_THREADS), fp64 and fp32 at N = 320 ... NMAX; a c N^3 fit per precision
with the N = 8192 / 16384 times EXTRAPOLATED (labelled so); and one run of the
reference's own CLI, `svd_cpu multicore 320 1 1 32` (BASELINE.json configs[0]).

usage: python tools/cpu_baseline.py [NMAX=2048] > gpurun_out/cpu_baseline.json
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
from splitmix import uniform_matrix  # noqa: E402
from bench import host_cpus  # noqa: E402


def main():
    nmax = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_fast.so"))
    L.ref_set_threads(threads)
    out = {"threads": threads, "host": host_cpus(), "band": 32,
           "library": "oracle/_ref/libref_fast.so (reference svd_parallel.h built from /root/reference sources)",
           "runs": {}}
    sizes = [n for n in (320, 640, 1024, 2048, 4096) if n <= nmax]
    for tname, dt, p1, p2 in (("f64", np.float64, L.ref_brd_p1_f64, L.ref_brd_p2_f64),
                              ("f32", np.float32, L.ref_brd_p1_f32, L.ref_brd_p2_f32)):
        pts = []
        for n in sizes:
            A = uniform_matrix(n, seed=n, lo=0.0, hi=5.0, dtype=np.float64).astype(dt)
            t0 = time.perf_counter()
            p1(A.ctypes.data_as(ctypes.c_void_p), n, 32)
            t1 = time.perf_counter()
            p2(A.ctypes.data_as(ctypes.c_void_p), n, 32)
            t2 = time.perf_counter()
            pts.append({"n": n, "stage1_s": round(t1 - t0, 3), "stage2_s": round(t2 - t1, 3),
                        "total_s": round(t2 - t0, 3), "gflops": round(8 / 3 * n ** 3 / (t2 - t0) / 1e9, 4)})
            print(f"{tname} n={n}: {t2 - t0:.2f} s", file=sys.stderr, flush=True)
        c = sum(p["total_s"] * p["n"] ** 3 for p in pts) / sum(float(p["n"]) ** 6 for p in pts)
        ext = {str(n): {"seconds": round(c * n ** 3, 1), "gflops": round(8 / 3 / c / 1e9, 4)} for n in (8192, 16384)}
        out["runs"][tname] = {"measured": pts, "fit_c_seconds_per_n3": c,
                              "extrapolated_NOT_measured": ext}
    exe = os.path.join(REPO, "oracle", "_ref", "svd_cpu")
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "data"))
        t0 = time.perf_counter()
        r = subprocess.run([exe, "multicore", "320", "1", "1", "32"], cwd=d, capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, OMP_NUM_THREADS=str(threads)))
        out["svd_cpu_multicore_320_1_1_32"] = {"rc": r.returncode, "wall_s": round(time.perf_counter() - t0, 2),
                                              "stdout": r.stdout[-1500:]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

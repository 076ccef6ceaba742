#!/usr/bin/env python3
"""Benchmark: two-stage bidiagonal reduction (dense -> band -> bidiagonal) on
MI355X, the metric of BASELINE.json:
    "GFLOP/s for two-stage bidiag reduction, N x N fp64, 1/2/4/8 MI355X"
counted as 8/3 N^3 flops per matrix (LAPACK GEBRD count).

One step = one full reduction (stage 1 + stage 2) of one synthetic N x N
matrix, uniform in [0,5) like the reference benchmark (svd_cuda_2.cu:1361),
already resident in HBM (one pristine copy per step is prepared before the
timed region, so no copy is timed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 8192] [--dtype f64] [--band 32]

N > 1: one process per GPU.  Launched by torch.distributed.run (WORLD_SIZE
set) it joins that job; run plainly as `python bench.py --gpus N` it starts
the N ranks itself (a torch.distributed.run child, before any GPU call) and
exits with their status (non-zero if fewer than N GPUs are visible).
Default (--mode dist): ONE N x N matrix per step (N = 16384, BASELINE.json
configs[4], unless --n is given), its stage 1 sharded over the N GPUs
(block-cyclic column panels, RCCL over xGMI, brd_ge2band_dist), the band of
matrix j gathered on rank j mod N, which runs its stage 2 (stage 2 stays
single-GPU, BASELINE.json north_star).  --mode replicas: every rank reduces
its own matrices (weak scaling).  The step time is the max over ranks and
`value` is the whole-job GFLOP/s.

What `value` measures (config.value_kind): the throughput of a STREAM of
independent reductions -- K matrices (default 20) issued back to back on L
stage-1 streams ("lanes", matrix j on lane j mod L; one GPU: K dealt in
balanced rounds of at most 10, plan_lanes) and ceil(L / 2) stage-2 streams
(matrix j's stage 2 on stream j mod that, after its stage 1, beside the
following matrices' stage 1; `--pipeline on`, the default), fill and drain
inside the timed region.  The same K steps one reduction at a
time on one lane (the reference's per-instance timing, timing.h:79-82) are
reported as `one_at_a_time`, and `latency_ms_per_reduction` is one matrix's
stage 1 + stage 2 under overlap.  After every timed region the library's
sticky stage-2 error words are read (brd_check_errors): a stalled sweep
fails the run instead of being timed.

Rank 0 prints ONE JSON line.  `value` comes from K timed steps with no
per-launch instrumentation; K more steps one at a time are then run with the
library's per-launch events (for the stage-1 apply stamped by the launch
itself, hipExtLaunchKernel) for the dominant kernel's roofline object.  Also
the CPU baseline: the reference's own tiled algorithm (built from its
sources by oracle/Makefile) timed on this host at N = 320, 640, 1024 (about
10-20 s) and 2048, extrapolated cubically from the largest sample to the GPU
problem size (labelled as such).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GFLOP/s for two-stage bidiag reduction, N×N fp64, 1/2/4/8 MI355X"
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}      # dense MFMA peaks (MI355X_MICROARCH.md / datasheet)
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    # --size is the spelling to use under torch.distributed.run, whose own
    # parser takes "--n" for an ambiguous abbreviation of its options
    p.add_argument("--size", "--n", dest="n", type=int, default=None,
                   help="matrix size (default 8192 on one GPU, BASELINE configs[2]; 16384 across GPUs, configs[4])")
    p.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    p.add_argument("--band", type=int, default=32)
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-n", type=str, default="320,640,1024,2048",
                   help="CPU-baseline sample sizes (comma separated; the largest is the reported sample)")
    p.add_argument("--s2", choices=["compat", "sigma"], default="compat",
                   help="stage-2 geometry: the reference's windows (the headline config) or the "
                        "sigma-preserving variant (BRD_SIGMA)")
    p.add_argument("--mode", choices=["dist", "replicas"], default="dist",
                   help="N > 1: sharded stage 1 of one matrix (dist) or independent replicas")
    p.add_argument("--pipeline", choices=["on", "off"], default="on",
                   help="on: stage 2 of matrix i runs on a second HIP stream beside stage 1 of "
                        "matrix i+1 (a stream of independent reductions); off: one reduction at a time")
    p.add_argument("--s2-cus", type=int, default=None,
                   help="pipelined: CUs reserved for stage 2 (default svdsolver_amd.overlap_cus(n))")
    p.add_argument("--one-at-a-time", choices=["on", "off"], default="on",
                   help="pipelined, one GPU: also time K steps without the overlap (reported as one_at_a_time)")
    p.add_argument("--lanes", type=int, default=None,
                   help="pipelined: stage-1 streams, matrix j on lane j mod L (default: one GPU plan_lanes(K), "
                        "10 for K = 20; across GPUs 8, each lane with its own RCCL communicator)")
    p.add_argument("--s2-lanes", type=int, default=None,
                   help="pipelined, one GPU: stage-2 streams (matrix j's stage 2 on stream j mod S2L; "
                        "default: one per lane)")
    p.add_argument("--pad", type=int, default=0,
                   help="leading dimension n + PAD elements for the device matrices")
    p.add_argument("--comm", choices=["rccl", "host"], default="rccl",
                   help="dist mode communicator: RCCL (one GPU per rank) or the host callback over gloo "
                        "(rehearsal of the multi-rank path with every rank on GPU 0)")
    p.add_argument("--stages", choices=["12", "1", "2"], default="12",
                   help="developer diagnostic: run only stage 1 or only stage 2 inside each step "
                        "(the line is then labelled, and is not the metric)")
    p.add_argument("--same-n", choices=["on", "off"], default="on",
                   help="N > 1 (dist): also time the one-GPU stream at the same size on rank 0 "
                        "(single_gpu_same_n in the line)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the distributed path even at world size 1 (launch through torch.distributed.run)")
    return p.parse_args()


def ensure_built():
    lib = os.path.join(REPO, "svdsolver_amd", "lib", "libbrd_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "svdsolver_amd")], check=True)


def host_cpus() -> dict:
    """What this host offers the CPU baseline: the CPUs this process may run on
    and the machine's physical core count (lscpu-equivalent from
    /proc/cpuinfo).  On the GPU box the job's CPU share is set by
    OMP_NUM_THREADS (16); os.cpu_count() shows the whole machine."""
    info = {"logical_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        cores = set()
        phys = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                cores.add((phys, core))
        if cores:
            info["physical_cores"] = len(cores)
    except OSError:
        pass
    return info


def cpu_baseline(sizes, band: int, gpu_n: int) -> dict:
    """The reference's tiled two-stage algorithm (parallel::brd_p1 +
    brd_p2<double>, svd_parallel.h:411/:640), built from
    the reference's sources by oracle/Makefile (README.md:32 flags minus
    -march=native), on n x n fp64 matrices uniform in [0,5), b = band, at each
    n in `sizes`.  OpenMP threads = the job's CPU share (OMP_NUM_THREADS, else
    the affinity set).  The EXTRAPOLATED time at the GPU problem size is cubic
    from the largest sample (not measured: ~40 min at 8192); a least-squares
    c n^3 + d n^2 fit over the samples is reported beside it.
    Falls back to the single-threaded C oracle (kind "port")."""
    import ctypes
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from splitmix import uniform_matrix
    hc = host_cpus()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or hc.get("affinity_cpus") or hc["logical_cpus"] or 1
    ref = os.path.join(REPO, "oracle", "_ref", "libref_fast.so")
    L = None
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        L.ref_set_threads(threads)
        kind, used = "reference", threads
    else:
        from oracle import oracle
        kind, used = "port", 1
    pts = []
    for n in sizes:
        A = uniform_matrix(n, seed=n, lo=0.0, hi=5.0, dtype=np.float64)
        t0 = time.perf_counter()
        if L is not None:
            L.ref_brd_p1_f64(A.ctypes.data_as(ctypes.c_void_p), n, band)
            L.ref_brd_p2_f64(A.ctypes.data_as(ctypes.c_void_p), n, band)
        else:
            oracle.brd_p2(oracle.brd_p1(A, band), band)
        pts.append((n, time.perf_counter() - t0))
    n_s, dt = pts[-1]
    # t = c n^3 + d n^2, least squares in relative error: at these sizes the
    # reference's time is dominated by its O(n^2) per-tile overheads and stage
    # 2 (320 -> 1024: t ~ n^2.1), so a pure c n^3 fit through the small sizes
    # overstates the large-n time ~2.5x (profiles/r02_cpu_baseline.json: this
    # fit over 320..1024 predicts 38.2 s at 2048, measured 37.3 s)
    M = np.array([[float(n) ** 3 / t, float(n) ** 2 / t] for n, t in pts])
    coef = np.linalg.lstsq(M, np.ones(len(pts)), rcond=None)[0] if len(pts) >= 2 else np.array([dt / n_s ** 3, 0.0])
    c, d = max(float(coef[0]), 0.0), max(float(coef[1]), 0.0)
    t_fit = c * float(gpu_n) ** 3 + d * float(gpu_n) ** 2
    # the reported extrapolation is CUBIC from the largest sample (VERDICT r5:
    # the fit's n^2 term flatters the CPU 2.3x per flop at 8192; SURVEY.md
    # section 6 measured the reference scaling cubically, 2048 -> 4096: 43.5 ->
    # 338.5 s); the fit is kept beside it for reference
    t_ext = dt * (float(gpu_n) / n_s) ** 3
    phys = hc.get("physical_cores")
    cores_note = (f"{used} OpenMP threads = the job's CPU share on this host (OMP_NUM_THREADS; the pool sizes "
                  f"a one-GPU job at 16 CPUs); the host has {phys} physical cores"
                  + (f": at ideal linear scaling over all of them the reference would reach "
                     f"{8.0 / 3.0 * n_s ** 3 / dt / 1e9 * phys / max(used, 1):.2f} GFLOP/s at n = {n_s} "
                     f"(an upper bound, not measured)" if phys and phys > used else ""))
    return {"value": round(8.0 / 3.0 * n_s ** 3 / dt / 1e9, 4), "unit": "GFLOP/s", "cores": used,
            "kind": kind, "sample": f"{n_s}x{n_s} fp64 two-stage reduction, b={band}, {dt:.2f} s, "
                                    f"{used} OpenMP threads",
            "threads": used, "host": hc, "cores_note": cores_note,
            "sizes_s": {str(n): round(t, 3) for n, t in pts},
            "extrapolated": {"n": gpu_n, "seconds": round(t_ext, 1),
                             "gflops": round(8.0 / 3.0 * gpu_n ** 3 / t_ext / 1e9, 4),
                             "basis": f"cubic from the largest sample (t({n_s}) * ({gpu_n}/{n_s})^3); NOT measured",
                             "fit_c_n3_d_n2": {"seconds": round(t_fit, 1),
                                               "gflops": round(8.0 / 3.0 * gpu_n ** 3 / t_fit / 1e9, 4),
                                               "basis": "least-squares over " + ",".join(str(n) for n, _ in pts)
                                                        + " (less conservative: its n^2 term dominates at these sizes)"}}}


def pmc_traffic(n: int, dtype: str, *kernel_prefixes: str):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC summary
    of THIS configuration, profiles/r*_pmc_n{n}_{dtype}.txt (tools/pmc.sh:
    separate FETCH_SIZE / WRITE_SIZE passes over the same bench command;
    FETCH_SIZE doubled for gfx950's 64-B tally of 128-B requests,
    MI355X_MICROARCH.md 'HBM').  The counters cannot be read inside this
    process, so the profile of the same command is the source; None when no
    summary of this configuration is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_n{n}_{dtype}.txt")))
    # the newest summary that has this kernel at all
    files = [f for f in files if any(ln.startswith(kernel_prefixes) for ln in open(f))]
    if not files:
        return None, None
    tot, cnt = 0.0, 0
    for line in open(files[-1]):
        if line.startswith(kernel_prefixes):
            f = line.split()
            try:
                d, two_fetch, wr = int(f[-4]), float(f[-2]), float(f[-1])
            except (ValueError, IndexError):
                continue
            tot += d * (two_fetch + wr) * 1024 * 1024
            cnt += d
    return (tot / cnt, os.path.relpath(files[-1], REPO)) if cnt else (None, None)


def apply_roofline(ap, dtype, n):
    """Stage-1 trailing update (k_apply, and k_apply_factor: the same apply with
    the next tree level's factor in one extra workgroup): per element of the
    trailing matrix one read + one write against 4b flops -> 8 flop/B at b = 32
    fp64, below the MFMA ridge (78.6 TF / 8 TB/s = 9.8 flop/B): HBM-bound."""
    ms, launches = ap["ms"], max(ap["launches"], 1)
    gbs = ap["bytes"] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    tf = ap["flops"] / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    tn = "double" if dtype == "f64" else "float"
    traffic, src = pmc_traffic(n, dtype, "void brd::k_apply<" + tn, "void brd::k_apply_factor<" + tn)
    return {"kernel": "k_apply + k_apply_factor (stage-1 trailing update, MFMA)", "bound": "hbm",
            "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
            "traffic": round(traffic) if traffic else None, "traffic_source": src,
            "algorithmic_bytes_per_launch": round(ap["bytes"] / launches),
            "achieved_tflops": round(tf, 3), "mfma_peak_tflops": PEAK_TFLOPS[dtype],
            "mfma_frac": round(tf / PEAK_TFLOPS[dtype], 4),
            "launches": ap["launches"], "avg_launch_us": round(ms * 1e3 / launches, 3),
            "flops_per_launch": round(ap["flops"] / launches)}


def pmc_mfma(n: int, dtype: str, kernel_prefix: str):
    """Counter-derived MFMA utilisation of a kernel from the committed
    rocprofv3 PMC summary of this configuration (tools/pmc.sh's MFMA pass:
    SQ_INSTS_VALU_MFMA_MOPS_F64/_F32 -- 512 flops per unit -- over
    SQ_BUSY_CYCLES x CUs x the per-CU-cycle MFMA peak); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_n{n}_{dtype}.txt")))
    if not files:
        return None
    for line in open(files[-1]):
        if line.startswith("MFMA " + kernel_prefix):
            try:
                return float(line.split()[-1])
            except ValueError:
                return None
    return None


def blkupd_roofline(bu, dtype, n):
    """Blocked stage 1's delayed trailing update (k_blkupd): C -= Lw RwT with
    K = 256 (the 4 panels' left and right block reflectors of a block), one
    read and one write of the trailing matrix per 128 columns against
    2 x 256 flops per element -> 32 flop/B fp64, above the MFMA ridge
    (78.6 TF / 8 TB/s = 9.8 flop/B): MFMA-bound."""
    ms, launches = bu["ms"], max(bu["launches"], 1)
    tf = bu["flops"] / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    gbs = bu["bytes"] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    tn = "double" if dtype == "f64" else "float"
    # the persistent kernel only (the default since round 4): an older summary
    # of the two-per-CU k_blkupd is another kernel's traffic
    traffic, src = pmc_traffic(n, dtype, "void brd::blk::k_blkupd_p<" + tn)
    return {"kernel": "k_blkupd / k_blkupd_p (stage-1 delayed rank-256 trailing update, MFMA)", "bound": "mfma",
            "achieved": round(tf, 3), "peak": PEAK_TFLOPS[dtype], "unit": "TFLOP/s",
            "frac": round(tf / PEAK_TFLOPS[dtype], 4),
            "traffic": round(traffic) if traffic else None, "traffic_source": src,
            "algorithmic_bytes_per_launch": round(bu["bytes"] / launches),
            "flops_per_launch": round(bu["flops"] / launches),
            "achieved_gbs": round(gbs, 1), "launches": bu["launches"],
            "avg_launch_us": round(ms * 1e3 / launches, 3),
            "mfma_util_counter": pmc_mfma(n, dtype, "k_blkupd")}


def rpass_roofline(rp, dtype, n):
    """Blocked stage 1's read passes (k_rpass: Y_j = A^T V_j and X_j = A U_j
    per panel, the split-K partial sums): the trailing matrix read once per
    pass, 2 x 32 flops per element -> 8 flop/B fp64: HBM-bound."""
    ms, launches = rp["ms"], max(rp["launches"], 1)
    gbs = rp["bytes"] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    tf = rp["flops"] / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    tn = "double" if dtype == "f64" else "float"
    traffic, src = pmc_traffic(n, dtype, "void brd::blk::k_rpass_d<" + tn)   # (the LDS-DMA pass, round 4 on)
    return {"kernel": "k_rpass / k_rpass_d (stage-1 read passes, MFMA)", "bound": "hbm", "achieved": round(gbs, 1),
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
            "traffic": round(traffic) if traffic else None, "traffic_source": src,
            "algorithmic_bytes_per_launch": round(rp["bytes"] / launches),
            "achieved_tflops": round(tf, 3), "launches": rp["launches"],
            "avg_launch_us": round(ms * 1e3 / launches, 3),
            "mfma_util_counter": pmc_mfma(n, dtype, "k_rpass")}


def stage2_roofline(sw, n, b, dtype, steps):
    """Stage 2 (k_sweeps, one launch per step): every bundle of sweeps
    streams the band rows below its first sweep in and out once (P = 3b
    elements per row), so the algorithmic HBM bytes are 2 * P * sizeof(T) *
    sum over bundles of the rows; the kernel is bound by its chain of
    dependent windows (about 4 per sweep), not by HBM (Stage 2)."""
    esz = 8 if dtype == "f64" else 4
    S = 3 if dtype == "f64" else 7      # sweeps per bundle (brd_stage2.hip sweeps_plan)
    P = 3 * b
    # minimum: the band (3b stored diagonals per row: the fill of a bulge
    # reaches b-1 below and 2b-1 above the diagonal) read once, written once
    minimum = 2.0 * n * P * esz
    # the design's volume: every bundle of S sweeps streams the rows below its
    # first sweep in and out of its LDS ring once
    rows = sum(n - i0 for i0 in range(0, n - 1, S))
    streamed = 2.0 * P * esz * rows
    # per launch (one launch per reduction; in the multi-GPU pipeline rank 0
    # runs the sweeps of only the matrices whose index is 0 mod world)
    ms = sw["ms"] / max(sw.get("launches", steps), 1)
    traffic, src = pmc_traffic(n, dtype, "void brd::k_sweeps<" + ("double" if dtype == "f64" else "float"))
    return {"kernel": "k_sweeps (stage-2 sweeps)", "bound": "latency (dependent window chain)",
            "ms": round(ms, 3),
            "minimum_bytes": round(minimum), "streamed_bytes_by_design": round(streamed),
            "traffic": round(traffic) if traffic else None, "traffic_source": src,
            "traffic_over_minimum": round(traffic / minimum, 1) if traffic else None,
            "hbm_gbs_streamed": round(streamed / (ms * 1e-3) / 1e9, 1) if ms > 0 else None,
            "windows": n * ((n // b) * 2),
            "us_per_sweep": round(ms * 1e3 / max(n - 1, 1), 3),
            "chain_bound_note": "about 4 dependent windows per sweep (lag-3 rule, DESIGN.md Stage 2)"}


def plan_lanes(k: int, lmax: int = 10) -> int:
    """Stage-1 lanes for a stream of k matrices: the fewest rounds that
    lmax lanes allow, but at least two (the first round's sweeps then run
    beside the second round's stage 1 instead of all at the end), dealt
    evenly (k = 20 -> 10 lanes x 2 rounds; 12 -> 6 x 2; 10 -> 5 x 2)."""
    rounds = max(2 if k >= 4 else 1, -(-k // lmax))
    return max(1, -(-k // rounds))


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def torchrun_cmd(gpus: int, argv, port: int) -> list:
    """The torch.distributed.run command that re-runs this script on `gpus`
    ranks with the same arguments ("--n" spelled "--size": the launcher's own
    parser reads "--n" as an ambiguous abbreviation of its options)."""
    fwd = ["--size" + a[3:] if a == "--n" or a.startswith("--n=") else a for a in argv]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + fwd


def maybe_spawn(args) -> None:
    """`python bench.py --gpus N` with no launcher around it: start the N ranks
    as a torch.distributed.run child (one process per GPU, rendezvous on
    127.0.0.1) and exit with its status.  Runs before this process touches
    the GPU (torch.cuda.device_count() does not initialise it on this image),
    so nothing here is exec'd from a GPU-initialised process."""
    if "WORLD_SIZE" in os.environ:
        w = int(os.environ["WORLD_SIZE"])
        if args.gpus != 1 and args.gpus != w:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={w}")
        return
    if args.gpus <= 1:
        return
    import torch
    ndev = torch.cuda.device_count()
    if ndev < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} requested but only {ndev} GPU(s) are visible")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = torchrun_cmd(args.gpus, sys.argv[1:], free_port())
    sys.exit(subprocess.call(cmd, env=env))


def single_gpu_same_n(S, torch, dev, n, b, tdt, steps, warmup, lanes, s2_cus, sigma):
    """The one-GPU stream of reductions at this n, timed on this rank alone
    (the same lanes / stage-2 reservation as the one-GPU bench): the
    denominator of a like-for-like multi-GPU efficiency at the multi-GPU
    default size."""
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    base = torch.rand((n, n), dtype=tdt, device=dev, generator=g) * 5.0
    mats = [base.clone() for _ in range(warmup + steps)]
    del base
    sa = [torch.cuda.Stream(dev) for _ in range(lanes)]
    sb = [torch.cuda.Stream(dev) for _ in range(lanes)]
    S.set_overlap(s2_cus)

    def issue(first, count):
        for i in range(count):
            j = first + i
            with torch.cuda.stream(sa[j % lanes]):
                S.ge2band(mats[j], b, sync=False)
                e1 = torch.cuda.Event()
                e1.record(sa[j % lanes])
            with torch.cuda.stream(sb[j % lanes]):
                sb[j % lanes].wait_event(e1)
                S.band2bd(mats[j], b, sigma=sigma, sync=False, extract=False)
    issue(0, warmup)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    issue(warmup, steps)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    S.check_errors()
    for s_ in sa + sb:
        S.release_stream(s_)
    del mats
    torch.cuda.empty_cache()
    return {"value": round(steps * 8.0 / 3.0 * n ** 3 / el / 1e9, 2), "ms_per_step": round(el / steps * 1e3, 3),
            "n": n, "lanes": lanes, "steps": steps}


def main():
    args = parse()
    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.gpus > 1 or args.force_dist
    if args.lanes is None:
        # one GPU: the K matrices dealt in balanced rounds over at most 10
        # stage-1 lanes (K = 20: 2 rounds of 10), so no round runs with part
        # of the lanes idle, and half as many stage-2 streams (a burst of
        # finished stage 1s queues there instead of taking 32 CUs each).
        # Same box, N = 8192 fp64, 20 steps: 8 lanes / 8 stage-2 streams (round
        # 5: 3+3+3+3+2+2+2+2 matrices) 25.12 / 25.08 TFLOP/s; 10 / 5 26.59 /
        # 26.73 / 26.70; 10 / 6 26.67; 10 / 4 26.06; 10 / 10 (24 CUs each)
        # 26.05; 12 / 6 26.15; 5 / 5 22.9; 20 / 8 25.8 (gpurun_out r6d / r6e,
        # profiles/r06_lanes_ab.txt).  Across GPUs: 8 lanes (one communicator each).
        args.lanes = (8 if multi else plan_lanes(args.steps)) if args.pipeline == "on" else 1
    if args.s2_lanes is None:
        args.s2_lanes = args.lanes if multi else max(1, (args.lanes + 1) // 2)
    # Every lane launches on two HIP streams; with the runtime's default of 4
    # hardware queues per process, streams beyond that share a queue and
    # their work serialises (measured: 2 lanes 14.1 -> 17.8 TFLOP/s once each
    # stream has a queue).  Read when the HIP runtime initialises, so set first;
    # raised (never lowered) from whatever the environment holds (4 on the
    # MI355X pool, HIP's own default).
    if args.lanes > 1:
        # (across GPUs every lane's stage-1 stream also carries an RCCL
        # communicator with internal streams of its own; giving them queues
        # too -- all 32 -- was measured slower at world size 1, N = 8192:
        # 11.95 vs 15.30 TFLOP/s distributed and 16.9 vs 21.1 single-GPU in
        # the same process, profiles/r04_hwq_ab.txt)
        want = min(32, args.lanes + args.s2_lanes + 4)
        try:
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
        except ValueError:
            have = 0
        if os.environ.get("BRD_BENCH_HWQ"):   # A/B: exactly this many (at most 32)
            os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, int(os.environ["BRD_BENCH_HWQ"])))
        elif have < want:
            os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    maybe_spawn(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_pg = world > 1 or args.force_dist
    if use_pg:
        if args.comm == "host":   # rehearsal: several ranks may share one GPU
            local = 0
            torch.cuda.set_device(local)
            dist.init_process_group("gloo", init_method="env://")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if rank == 0 or world == 1:
        ensure_built()
    if world > 1:
        dist.barrier()
    import svdsolver_amd as S

    n, b = args.n, args.band
    if n is None:
        n = 8192 if world == 1 else 16384   # BASELINE.json configs[2] / configs[4]
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    dist_mode = (world > 1 or args.force_dist) and args.mode == "dist"
    pipelined = args.pipeline == "on"
    serial_too = pipelined and not dist_mode and args.one_at_a_time == "on"   # also time them one at a time
    # warmup, the timed steps, the profiled steps (+ the one-at-a-time steps)
    nmat = args.warmup + (3 if serial_too else 2) * args.steps
    mode = {"pipe": pipelined}
    s2_cus = S.overlap_cus(n) if pipelined else 0
    if args.s2_cus is not None:
        s2_cus = args.s2_cus
    lanes = args.lanes if pipelined else 1
    s2_lanes = (args.s2_lanes if not dist_mode else lanes) if pipelined else 1
    if pipelined and s2_lanes * max(s2_cus, 1) > torch.cuda.get_device_properties(dev).multi_processor_count:
        # every stage-2 stream's kernel is a persistent grid of s2_cus
        # workgroups, one per CU: together they must fit the chip
        sys.exit(f"bench.py: stage-2 streams * s2_cus = {s2_lanes} * {s2_cus} exceeds the device's CUs")
    S.set_overlap(s2_cus)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    # Two launch streams per lane: stage 1 (and the band gather) on s_a, stage 2
    # on s_b.  Pipelined, stage 2 of matrix i waits only for stage 1 of matrix
    # i, so it runs beside stage 1 of the lane's next matrix (stage 2 is a
    # latency-bound chain on a few dozen CUs, stage 1 HBM-bound on the rest);
    # otherwise s_b's work is ordered after all of s_a's and vice versa (one
    # reduction at a time).  L lanes side by side (default 8), matrix j on lane
    # j mod L (the library keeps a workspace -- and, across GPUs, an RCCL
    # communicator -- per launch stream), so one lane's latency-bound work
    # (leaf factors, tail panels, the stage-2 chase, the distributed panel
    # loop's collectives) overlaps another lane's HBM-bound trailing updates.
    # Measured at N = 8192 fp64 (20 steps, one hardware queue per stream):
    # L = 1 14.1 TFLOP/s, L = 2 18.2, L = 4 19.9, L = 8 20.3; again this round
    # 4 vs 8: 19.78 vs 20.13 on one GPU and, through the distributed path at
    # world size 1 over RCCL (--force-dist, 12 steps), 14.6 vs 16.0 -- across
    # GPUs a matrix's stage 1 is a chain of per-panel collectives and factors,
    # so more matrices in flight hide more of it.
    sa_l = [torch.cuda.Stream(dev) for _ in range(lanes)]
    sb_l = [torch.cuda.Stream(dev) for _ in range(s2_lanes)]
    if dist_mode:
        from svdsolver_amd import dist as D
        for s_a in sa_l:   # one communicator per lane's stage-1 stream
            if args.comm == "host":
                D.init_host(stream=s_a)
            else:
                D.init_rccl(stream=s_a)
        n_loc = D.local_cols(n, b, world, rank)
        base = torch.rand((n, max(n_loc, 1)), dtype=tdt, device=dev, generator=g)[:, :n_loc] * 5.0
        mats = [base.contiguous().clone() for _ in range(nmat)]
        # Matrix j's band goes to rank j mod world, which runs its stage 2; two
        # band buffers per lane and rank so a gather never lands in a band whose
        # sweep may still be running (the stage-1 stream also waits for that
        # sweep).
        nbuf = 2 if pipelined else 1

        def root_of(j):
            return j % world if pipelined else 0

        def band_of(j):
            return j % lanes, (j // lanes) % nbuf

        # only the band buffers this rank roots, allocated before any timed
        # region (with 8 lanes over 8 ranks: lane r's two buffers on rank r,
        # 4 GB at N = 16384 instead of 32 GB; 8 host-callback ranks sharing
        # one GPU would not fit otherwise)
        Bfull = {key: torch.empty((n, n), dtype=tdt, device=dev)
                 for key in sorted({band_of(j) for j in range(nmat) if root_of(j) == rank})}
        s2_done = {key: None for key in Bfull}

        def stage1(A, j):
            D.ge2band(A, n, b, sync=False)
            r, key = root_of(j), band_of(j)
            if rank == r and s2_done[key] is not None:
                torch.cuda.current_stream(dev).wait_event(s2_done[key])
            D.gather_band(A, n, b, root=r, out=Bfull[key] if rank == r else None, sync=False)

        def stage2(A, j):
            if rank == root_of(j):
                key = band_of(j)
                S.band2bd(Bfull[key], b, sigma=args.s2 == "sigma", sync=False, extract=False)
                e = torch.cuda.Event()
                e.record(torch.cuda.current_stream(dev))
                s2_done[key] = e
    else:
        base = torch.rand((n, n), dtype=tdt, device=dev, generator=g) * 5.0
        mats = []
        for _ in range(nmat):
            M = torch.empty((n, n + args.pad), dtype=tdt, device=dev)[:, :n]
            M.copy_(base)
            mats.append(M)

        def stage1(A, j):
            if args.stages != "2":
                S.ge2band(A, b, sync=False)

        def stage2(A, j):
            if args.stages != "1":
                S.band2bd(A, b, sigma=args.s2 == "sigma", sync=False, extract=False)
    del base


    def issue(first, count, ev=None):
        last = None
        # one reduction at a time: lane 0 only.  Matrices queued on the other
        # lanes' streams would sit behind cross-stream barriers, and queues
        # parked on barriers slow the dispatch of the active one (measured:
        # stage 1 137 ms vs 89 ms with 4 lanes' streams waiting).
        nl = lanes if mode["pipe"] else 1
        for i in range(count):
            j = first + i
            A = mats[j]
            s_a, s_b = sa_l[j % nl], sb_l[j % (s2_lanes if mode["pipe"] else 1)]
            with torch.cuda.stream(s_a):
                if not mode["pipe"] and last is not None:
                    s_a.wait_event(last)
                if ev:
                    ev[i][0].record(s_a)
                stage1(A, j)
                e1 = torch.cuda.Event(enable_timing=bool(ev))
                e1.record(s_a)
            with torch.cuda.stream(s_b):
                s_b.wait_event(e1)
                if ev:
                    ev[i][1].record(s_b)
                stage2(A, j)
                last = torch.cuda.Event(enable_timing=bool(ev))
                last.record(s_b)
                if ev:
                    ev[i][2] = (e1, last)

    issue(0, args.warmup)
    torch.cuda.synchronize(dev)
    S.check_errors()

    host_issue_ms = []

    def run_steps(first):
        """K steps bracketed by barrier + synchronize; per-step stage split by
        events on the launch stream.  Returns (elapsed, stage1 ms, stage2 ms)."""
        ev = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), None]
              for _ in range(args.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        issue(first, args.steps, ev)
        host_issue_ms.append(1e3 * (time.perf_counter() - t0))   # the host's launch calls (diagnostic)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        # a stage-2 sweep that gave up waiting (sticky error word) fails the
        # run rather than being timed as a valid reduction
        S.check_errors()
        s2 = [e[1].elapsed_time(e[2][1]) for i, e in enumerate(ev) if not dist_mode or rank == root_of(first + i)]
        return (el, sum(e[0].elapsed_time(e[2][0]) for e in ev) / args.steps,
                sum(s2) / max(1, len(s2)))

    # (1) the timed steps: `value` (no per-launch instrumentation inside)
    elapsed, s1, s2 = run_steps(args.warmup)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.comm == "rccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    one_at_a_time = None
    if serial_too:
        # (2) the same kind of steps without any overlap (one reduction at a
        # time, whole chip per stage): the latency of one reduction, reported
        # beside the stream's throughput
        mode["pipe"] = False
        S.set_overlap(0)
        el_s, s1_s, s2_s = run_steps(args.warmup + args.steps)
        one_at_a_time = {"value": round(args.steps * 8.0 / 3.0 * n ** 3 / el_s / 1e9, 2),
                         "ms_per_step": round(el_s / args.steps * 1e3, 3),
                         "stage_ms": {"stage1": round(s1_s, 3), "stage2": round(s2_s, 3)}}
    # (3) K steps with the library's per-launch HIP events on its launch
    # streams: kernel durations for the roofline object.  On one GPU they run
    # one reduction at a time (as in (2)), so a kernel's duration is its own,
    # not stretched by the concurrent lanes of (1); across GPUs they repeat (1).
    S.profile_reset()
    S.profile_enable(True)
    el_prof, _, _ = run_steps(args.warmup + (2 if serial_too else 1) * args.steps)
    S.profile_enable(False)
    if serial_too:
        S.set_overlap(s2_cus)
        mode["pipe"] = True
    ap = S.profile_query("s1_apply")
    fa = S.profile_query("s1_factor")
    sw = S.profile_query("s2_sweep")
    bu = S.profile_query("s1_blkupd")
    rp = S.profile_query("s1_rpass")
    cq = S.profile_query("s1_cqr")
    pp = S.profile_query("s1_prep")
    cm = S.profile_query("s1_comm")   # the distributed blocked path's data movement around its collectives
    blocked = bu["launches"] > 0

    flops_per = 8.0 / 3.0 * n ** 3
    matrices = 1 if (world == 1 or dist_mode) else world   # matrices reduced per step, whole job
    value = matrices * args.steps * flops_per / elapsed / 1e9
    # across GPUs: the one-GPU stream at the same n on rank 0 (the others wait),
    # so the line carries a like-for-like 1 -> N efficiency at this size
    same_n = None
    rehearse = os.environ.get("BRD_BENCH_SAME_N") == "1"   # world-1 rehearsal (--force-dist)
    if (world > 1 or rehearse) and dist_mode and args.comm == "rccl" and args.same_n == "on":
        if rank == 0:
            try:
                same_n = single_gpu_same_n(S, torch, dev, n, b, tdt, args.steps, max(1, args.warmup), lanes,
                                           S.overlap_cus(n), args.s2 == "sigma")
            except Exception as e:   # reported, never fatal to the multi-GPU line
                same_n = {"value": None, "error": str(e)[:200]}
        dist.barrier()
    if rank == 0:
        out = {
            "metric": METRIC if args.stages == "12" else f"DIAGNOSTIC stage {args.stages} only (not the metric)",
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if (world > 1 and not dist_mode) else "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic uniform [0,5) N x N, resident in HBM",
            "config": {"workload": (f"stream of independent two-stage bidiagonal reductions {n}x{n} {args.dtype}"
                                    if pipelined else f"two-stage bidiagonal reduction {n}x{n} {args.dtype}, one at a time")
                                   + f", band {b}, "
                                   + ("stage 2 = reference window geometry (compat)" if args.s2 == "compat"
                                      else "stage 2 = sigma-preserving geometry (BRD_SIGMA)"),
                       "value_kind": (("stream throughput: K independent matrices issued back to back, each one's "
                                       f"stage 1 sharded over the {world} ranks, its band gathered on rank j mod "
                                       f"{world}, whose stage 2 runs beside the following matrices' stage 1; fill "
                                       "and drain inside the timed region" if dist_mode else
                                       f"stream throughput: K independent matrices issued back to back on {lanes} "
                                       f"stage-1 stream(s) (matrix j on lane j mod {lanes}) and {s2_lanes} stage-2 "
                                       f"stream(s) (matrix j's stage 2 on stream j mod {s2_lanes}, after its stage 1, "
                                       "beside the following matrices' stage 1), fill and drain inside the timed region; "
                                       "per-reduction latency under overlap: latency_ms_per_reduction; one reduction "
                                       "at a time: one_at_a_time") if pipelined else "one reduction at a time"),
                       "n": n, "band": b,
                       # matrices in flight at once: one per lane in the stream
                       "global_batch": matrices * (lanes if pipelined else 1),
                       "matrices_per_timed_region": matrices * args.steps,
                       "parallelism": (f"stage1 block-cyclic columns over {world} GPUs ({'RCCL' if args.comm == 'rccl' else 'host gloo'}), stage2 on rank "
                                       + ("(matrix index mod world)" if pipelined else "0")
                                       if dist_mode else f"replicas{world}"),
                       "pipeline": ("stage 2 of matrix i on a second HIP stream beside stage 1 of matrix i+1"
                                    if pipelined else "off: one reduction at a time"),
                       "stage2_cus": s2_cus or "all", "lanes": lanes, "stage2_streams": s2_lanes,
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "rccl_nranks": world if (dist_mode and args.comm == "rccl") else None},
            "latency_ms_per_reduction": round(s1 + s2, 3),
            # host time to issue the K steps' launches: the timed pass (, one at a time, profiled)
            "host_issue_ms": [round(x, 1) for x in host_issue_ms],
            "one_at_a_time": one_at_a_time,
            "stage_ms": {"stage1": round(s1, 3), "stage2": round(s2, 3)},
            "profiled_ms_per_step": round(el_prof / args.steps * 1e3, 3),
            "profiled_pass": "one reduction at a time" if serial_too else "as the timed steps",
            # the dominant stage-1 kernel: the blocked path's delayed update
            # (k_blkupd, MFMA-bound) when it ran, else the per-panel apply
            "roofline": blkupd_roofline(bu, args.dtype, n) if blocked else apply_roofline(ap, args.dtype, n),
            "roofline_read_pass": rpass_roofline(rp, args.dtype, n) if blocked else None,
            "roofline_tail_apply": apply_roofline(ap, args.dtype, n) if blocked and ap["launches"] else None,
            "stage2": stage2_roofline(sw, n, b, args.dtype, args.steps),
            "kernel_ms_per_step": {"s1_blkupd": round(bu["ms"] / args.steps, 3),
                                   "s1_rpass": round(rp["ms"] / args.steps, 3),
                                   "s1_panel_cqr": round(cq["ms"] / args.steps, 3),
                                   "s1_prep": round(pp["ms"] / args.steps, 3),
                                   "s1_comm": round(cm["ms"] / args.steps, 3),
                                   "s1_apply": round(ap["ms"] / args.steps, 3),
                                   "s1_factor": round(fa["ms"] / args.steps, 3),
                                   "s2_sweep": round(sw["ms"] / args.steps, 3)},
            "stage1_path": "blocked (delayed two-sided update, brd_stage1_blk.hip) + per-panel tail" if blocked
                           else "per-panel (brd_stage1.hip)",
        }
        if same_n is not None:
            out["single_gpu_same_n"] = same_n
            out["efficiency_vs_single_gpu_same_n"] = (round(value / (world * same_n["value"]), 4)
                                                      if same_n.get("value") else None)
        if args.cpu_baseline == "auto":
            try:
                out["cpu_baseline"] = cpu_baseline([int(x) for x in args.cpu_n.split(",")], b, n)
            except Exception as e:   # the baseline is reported, never required
                out["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
        print(json.dumps(out), flush=True)
    if dist_mode:
        D.finalize()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""bench.py's launcher contract on a host without GPUs (CPU suite): asked for
N > 1 GPUs without an external launcher it must refuse loudly -- never run a
silent one-GPU measurement under an N-GPU label (What's missing
item 4)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_more_gpus_than_visible():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert "requested but only" in out.stderr


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "1"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


def test_torchrun_command_passes_size_through():
    """`python bench.py --gpus N --n 16384`: the spawned torch.distributed.run
    must hand every bench argument to the script (its own parser would take
    "--n" as an ambiguous abbreviation of --nnodes / --nproc-per-node ...)."""
    import importlib.util
    from torch.distributed.run import get_args_parser
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cmd = bench.torchrun_cmd(2, ["--gpus", "2", "--n", "4096", "--steps", "3", "--warmup", "1"], 29999)
    ns = get_args_parser().parse_args(cmd[3:])
    assert ns.nproc_per_node == "2" and ns.training_script.endswith("bench.py")
    assert ns.training_script_args == ["--gpus", "2", "--size", "4096", "--steps", "3", "--warmup", "1"]


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.gpu
def test_bench_two_ranks_end_to_end():
    """The driver's N > 1 bench path, end to end on one GPU: two ranks under
    torch.distributed.run, stage 1 sharded over them, bands gathered on rank
    j mod 2, stage 2 beside the next matrices, the lanes' communicators --
    through the host-callback communicator (RCCL needs one GPU per rank).
    Rank 0 prints one JSON line with n_gpus = 2 and a positive value."""
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--comm", "host", "--size", "1024", "--steps", "3", "--warmup", "1",
           "--lanes", "2", "--cpu-baseline", "off"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["n"] == 1024
    assert d["config"]["matrices_per_timed_region"] == 3


@pytest.mark.gpu
def test_bench_eight_ranks_end_to_end():
    """bench.py --gpus 8 as the driver launches it on an 8-GPU node (configs[4]'s
    P = 8 layout: 8 ranks x the lanes' communicators), rehearsed on one GPU
    through the host-callback communicator at n = 2048 (the blocked path with
    the sharded row-panel CholeskyQR)."""
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "8", "--comm", "host", "--size", "2048", "--steps", "2", "--warmup", "1",
           "--lanes", "2", "--cpu-baseline", "off"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["value"] > 0 and d["config"]["n"] == 2048
    assert d["config"]["matrices_per_timed_region"] == 2

"""bench.py's launcher contract on a host without GPUs (CPU suite): asked for
N > 1 GPUs without an external launcher it must refuse loudly -- never run a
silent one-GPU measurement under an N-GPU label (What's missing
item 4)."""
import os
import subprocess
import sys

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

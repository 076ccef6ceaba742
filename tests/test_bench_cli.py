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

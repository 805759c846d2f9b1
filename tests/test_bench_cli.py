"""bench.py's command line: --gpus N means N ranks (one per GPU).

Run without a launcher and N > 1, bench.py starts itself under torch.distributed.run as a child
process; under a launcher WORLD_SIZE must equal --gpus.  CPU-only checks (no rank is started)."""
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 8])
def test_rank_launch_command(n):
    argv = ["--gpus", str(n), "--steps", "20", "--warmup", "5"]
    cmd = bench.rank_launch_cmd(argv, n, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == str(n)
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert "--nnodes=1" in cmd
    script = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[script + 1:] == argv  # the ranks get the same arguments


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=300)


def test_gpus_more_than_visible_fails_loudly():
    # this container has no GPU (the 1-GPU box has one): --gpus 2 must not time a single rank
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "1"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_latency_modes_are_single_gpu():
    r = _run(["--gpus", "2", "--mode", "dropin"])
    assert r.returncode != 0 and "single-GPU" in r.stderr

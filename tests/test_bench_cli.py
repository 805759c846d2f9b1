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


def test_line_reports_what_bounds_the_kernel():
    """The JSON line's fields, from stubbed measurements (no GPU): the metric's HBM roofline with
    the PMC traffic's own fraction of the peak, the FP64 VALU binding roofline, the hit-order
    gain of the same run and the single-plan (one isolated batch) rate."""
    args = bench.parse(["--steps", "20", "--warmup", "5"])
    ctx = dict(kind="sspp", kernel_name="k_sspp_c2f")
    B, kernel_s, per_launch = 4096, 50e-6, 20 * 4096
    line = bench.bench_line(args, ctx, dict(workload="stub"), 1, 4, True, B, elapsed=70e-6, enqueue_s=5e-6,
                            kernel_s=kernel_s, bytes_per=569, flops_per=537056, per_launch=per_launch,
                            traffic=2.4e6, traffic_src="stub", exec_per=7443.0, exec_src="stub", cpu=None,
                            extras={"isolated_step_us": 25.0, "order1_elapsed_s": 77e-6})
    assert line["value"] == pytest.approx(20 * B / 70e-6)
    r = line["roofline"]
    assert r["bound"] == "hbm" and r["frac"] == pytest.approx(569 * per_launch / kernel_s / 8e12)
    assert r["traffic_frac"] == pytest.approx(2.4e6 / kernel_s / 8e12)
    b = line["binding_roofline"]
    assert b["bound"] == "fp64_valu" and b["frac"] == pytest.approx(7443.0 * per_launch / kernel_s / 78.6e12)
    assert line["config"]["order_gain"] == pytest.approx(77 / 70)
    assert line["single_plan_cand_per_s"] == pytest.approx(B / 25e-6)
    assert line["isolated_step_us"] == 25.0
    # with the PMC issue record the binding resource is VALU issue, the FP64 figure beside it
    line = bench.bench_line(args, ctx, dict(workload="stub"), 1, 4, True, B, 70e-6, 5e-6, kernel_s, 569, 537056,
                            per_launch, 2.4e6, "stub", 1786.0, "stub", None,
                            {"valu_issue": {"per_simd": 0.49, "occupancy": 10.1, "source": "stub"}})
    b = line["binding_roofline"]
    assert b["bound"] == "valu_issue" and b["frac"] == 0.49 and b["mean_occupancy_waves_per_cu"] == 10.1
    assert b["fp64_valu"]["frac"] == pytest.approx(1786.0 * per_launch / kernel_s / 78.6e12)
    # without PMC records or the extra runs the fields are absent or null, never invented
    line = bench.bench_line(args, ctx, {}, 2, 4, True, B, 70e-6, 5e-6, kernel_s, 569, 537056, per_launch,
                            None, None, None, None, None, {})
    assert line["roofline"]["traffic_frac"] is None and line["binding_roofline"]["frac"] is None
    assert "order_gain" not in line["config"] and "single_plan_cand_per_s" not in line
    assert line["n_gpus"] == line["ranks_joined"] == 2

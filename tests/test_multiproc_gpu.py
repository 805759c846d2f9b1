"""The real multi-rank exchange in separate processes.

Two (and, for the step protocol, four) processes share cuda:0 and form a gloo group (device records are staged through host
memory by sspp_amd.all_gather_records; RCCL itself is exercised only on the driver's 8-GPU
node).  Everything else is the production path:
* bench.native_runner: executor launches on two streams, the chunk's per-step argmin records
  all-gathered once, reduce_best_steps on the device — per-step global records must be
  bit-identical to one rank scoring the union of the shards (world * B candidates per step);
* CesPlanner.step with world = 2 driven on a non-default stream (pack, gather, unpack ordered
  on that stream) — every rank's distribution, elites and best must be bit-identical to the
  single-rank planner's, iteration by iteration.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, mode, world, batch=0):
    port = _free_port()
    outs = [str(tmp_path / ("%s_w%d_r%d.json" % (mode, world, r))) for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, WORKER, mode, str(world), str(r), str(port), outs[r],
                               str(batch)], env=env) for r in range(world)]
    try:
        for p in procs:
            assert p.wait(timeout=200) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [json.load(open(o)) for o in outs]


@pytest.mark.timeout(450)
@pytest.mark.parametrize("world", [2, 4])
def test_bench_step_protocol_ranks_equal_one(cuda, tmp_path, world):
    many = _run(tmp_path, "steps", world, batch=4096 // world)
    one = _run(tmp_path, "steps", 1, batch=4096)  # the union of the shards per step
    for r in range(1, world):
        assert many[r]["records"] == many[0]["records"]
    assert many[0]["records"] == one[0]["records"]
    assert sum(len(c) for c in one[0]["records"]) == 30


@pytest.mark.timeout(450)
def test_ces_two_ranks_non_default_stream_equals_one(cuda, tmp_path):
    two = _run(tmp_path, "ces", 2)
    one = _run(tmp_path, "ces", 1)
    assert two[0]["iterations"] == two[1]["iterations"] == one[0]["iterations"]
    assert any(it["n_success"] > 0 for it in one[0]["iterations"])

"""Multi-rank sharding of the candidate batch, world_size 2 on gloo (CPU).

Each rank scores candidates with global ids [r*B/R, (r+1)*B/R) (counter-based Philox keyed by
the global id), reduces its shard to one record, and the records are all-gathered and reduced
with the product's reducer (lowest cost, lowest global id on ties).  The result must equal the
single-process argmin over the whole batch — the property the RCCL path in bench.py relies on.
Scoring here is the oracle (CPU); the GPU path is the same reduction over device records.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import SCENES

W_, B_ = 40, 96


def _problem():
    from oracle import mjcf_ref
    from oracle import oracle as O
    m = mjcf_ref.load(os.path.join(SCENES, "robocrane.xml"))
    start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
    u = np.array([i / 9 for i in range(10)])
    knots, ctrl0 = O.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
    return O.Scene(m, 0, 7), knots, ctrl0


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    import sspp_amd as S
    scene, knots, ctrl0 = _problem()
    per = B_ // world
    first = rank * per
    ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), 11, first, per)
    arc, feas = O.sspp_score(scene, knots, 3, ctrl, W_, nthreads=1)
    idx, cost = O.argmin(arc, feas)
    rec = torch.tensor([np.float64(cost).view(np.int64), idx + first if idx >= 0 else -1,
                        int(feas.sum()), 0], dtype=torch.int64)
    out = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, rec)
    parts = [(float(np.int64(o[0].item()).view(np.float64)), int(o[1]), int(o[2])) for o in out]
    q.put((rank, S.reduce_best(parts)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_argmin_equals_global(world):
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scene, knots, ctrl0 = _problem()
    ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), 11, 0, B_)
    arc, feas = O.sspp_score(scene, knots, 3, ctrl, W_, nthreads=1)
    idx, cost = O.argmin(arc, feas)
    assert feas.any() and not feas.all()
    for r in range(world):
        assert res[r] == (cost, idx, int(feas.sum()))


def test_bench_ids_are_disjoint():
    """bench.py: step i on rank r scores ids [(i*world + r)*B, +B) -> no overlap, no gaps."""
    for world in (1, 2, 4, 8):
        B = 16
        ids = sorted(x for i in range(3) for r in range(world)
                     for x in range((i * world + r) * B, (i * world + r + 1) * B))
        assert ids == list(range(3 * world * B))

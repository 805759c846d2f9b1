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


# Philox seed of the sampled batch: chosen so that the batch mixes feasible and infeasible
# candidates (asserted in the test; round 2 moved it from 11 when the sampler changed and the
# old seed's batch became all-infeasible)
SEED = 12


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    import sspp_amd as S
    scene, knots, ctrl0 = _problem()
    per = B_ // world
    first = rank * per
    ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), SEED, first, per)
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
    ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), SEED, 0, B_)
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


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from sspp_amd.runtime import all_gather_records
    # bench.py's chunk records [G][4] -> [world][G][4]; CesPlanner's flat slot records
    rec = torch.arange(12 * 4, dtype=torch.int64).view(12, 4) + 1000 * rank
    out = torch.empty((world, 12, 4), dtype=torch.int64)
    all_gather_records(out, rec)
    flat = torch.arange(10, dtype=torch.float64) + 0.5 * rank
    fout = torch.empty(10 * world, dtype=torch.float64)
    all_gather_records(fout, flat)
    q.put((rank, out.tolist(), fout.tolist()))
    dist.destroy_process_group()


def test_all_gather_records_gloo_layout():
    """sspp_amd.all_gather_records on a gloo group (the host-staged path) lays the ranks'
    records out exactly as RCCL's all_gather_into_tensor does: rank-major."""
    import torch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.stack([torch.arange(48, dtype=torch.int64).view(12, 4) + 1000 * r for r in range(world)])
    wantf = torch.cat([torch.arange(10, dtype=torch.float64) + 0.5 * r for r in range(world)])
    for r in range(world):
        assert res[r][0] == want.tolist() and res[r][1] == wantf.tolist()


G_ = 3  # steps per chunk (bench.native_runner gathers a chunk's per-step records at once)


def _steps_worker(rank, world, port, q, per):
    """bench.native_runner's protocol on gloo: G_ steps, step t scoring ids (t*world + rank)*per
    + [0, per); the chunk's per-step records [G][4] all-gathered once -> [world][G][4]."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    import sspp_amd as S
    from sspp_amd.runtime import all_gather_records
    scene, knots, ctrl0 = _problem()
    recs = []
    for t in range(G_):
        first = (t * world + rank) * per
        ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), SEED, first, per)
        arc, feas = O.sspp_score(scene, knots, 3, ctrl, W_, nthreads=1)
        idx, cost = O.argmin(arc, feas)
        recs.append([int(np.float64(cost).view(np.int64)), idx + first if idx >= 0 else -1, int(feas.sum()), 0])
    rec = torch.tensor(recs, dtype=torch.int64)
    out = torch.empty((world, G_, 4), dtype=torch.int64)
    all_gather_records(out, rec)
    steps = []
    for t in range(G_):  # the per-step reduction reduce_best_steps runs on the device
        parts = [(float(np.int64(out[r, t, 0].item()).view(np.float64)), int(out[r, t, 1]), int(out[r, t, 2]))
                 for r in range(world)]
        steps.append(S.reduce_best(parts))
    q.put((rank, steps, out.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [4])
def test_chunked_step_records_four_ranks(world):
    """The 4-rank layout of the driver's SCALE run, rehearsed on gloo: every rank's chunk of
    per-step records gathers rank-major, and each step's reduced record equals one rank scoring
    that step's whole batch (world * per candidates, ids t * world * per + [0, world * per))."""
    from oracle import oracle as O
    per = 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + os.getpid() % 1000
    procs = [ctx.Process(target=_steps_worker, args=(r, world, port, q, per)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (s, g)) for r, s, g in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scene, knots, ctrl0 = _problem()
    B = world * per
    some_mixed = False
    for t in range(G_):
        ctrl = O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), SEED, t * B, B)
        arc, feas = O.sspp_score(scene, knots, 3, ctrl, W_, nthreads=1)
        idx, cost = O.argmin(arc, feas)
        some_mixed |= bool(feas.any() and not feas.all())
        want = (cost, idx + t * B if idx >= 0 else -1, int(feas.sum()))
        for r in range(world):
            assert res[r][0][t] == want
    assert some_mixed
    for r in range(1, world):  # every rank holds the same gathered records
        assert res[r][1] == res[0][1]


def test_host_reducer_ties_go_to_lowest_id():
    """Equal costs on several ranks: the lowest global id wins, whatever the rank order."""
    import sspp_amd as S
    parts = [(1.5, 900, 2), (1.5, 17, 1), (float("inf"), -1, 0), (2.0, 3, 4)]
    assert S.reduce_best(parts) == (1.5, 17, 7)
    assert S.reduce_best(parts[::-1]) == (1.5, 17, 7)
    assert S.reduce_best([(float("inf"), -1, 0)] * 4) == (float("inf"), -1, 0)

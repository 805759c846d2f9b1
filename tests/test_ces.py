"""TaskSpacePlanner CES iteration (include/sspp/tsp_planner.h:72-145): oracle vs a literal
restatement of the reference, and the device planner (sspp_ces_*, `_tsp`) vs the oracle.

Bars: elite sets, best slots and success counts identical; the distribution after each update
bit-identical to the oracle run on the same candidate results (both sum in the canonical wave
order), and within 1e-12 of the reference's sequential summation order.
"""
import math
import os

import numpy as np
import pytest

from oracle import mjcf_ref
from oracle import oracle as O
from tests.conftest import SCENES

STACKING = os.path.join(SCENES, "stacking.xml")
ROBOCRANE = os.path.join(SCENES, "robocrane.xml")
LO, HI = (-0.5, -0.5, 0.0, -1.6), (0.5, 0.5, 0.6, 1.6)


def literal_update(cost, status, vias, mean, sigma, frac=0.3, inc=1.5, dec=0.95, sigma_floor=0.0,
                   var_beta=0.2, mean_lr=0.5, sd_min=0.01, sd_max=0.5, dist_z_min=0.3,
                   lo=(-2.0,) * 4, hi=(2.0,) * 4):
    """tsp_planner.h:121-142 / tsp_elites.h / tsp_distribution.h transcribed with Python
    floats (sequential sums, math.log = glibc log); successes in slot order, ties -> low slot."""
    succ = [i for i in range(len(cost)) if status[i]]
    mean, sigma = [list(r) for r in mean], [list(r) for r in sigma]

    def clampsd(s):
        return max(min(max(s, sd_min), sd_max), sigma_floor)
    if not succ:
        return [[clampsd(s * inc) for s in r] for r in sigma], mean, None, []
    k = max(1, int(len(succ) * frac))
    el = sorted(succ, key=lambda i: (cost[i], i))[:k]
    w = [math.log(k + 0.5) - math.log(i + 1.0) for i in range(k)]
    sw = 0.0
    for x in w:
        sw += x
    w = [x / sw for x in w]
    K = len(mean)
    for i in range(K):
        em = [0.0] * 4
        for j in range(k):
            for d in range(4):
                em[d] += w[j] * vias[el[j]][i][d]
        nm = [mean[i][d] + mean_lr * (em[d] - mean[i][d]) for d in range(4)]
        nm[2] = max(nm[2], dist_z_min)
        nm = [lo[d] if nm[d] < lo[d] else (hi[d] if hi[d] < nm[d] else nm[d]) for d in range(4)]
        mean[i] = nm
        ve = [0.0] * 4
        for j in range(k):
            diff = [vias[el[j]][i][d] - nm[d] for d in range(4)]
            if lo[3] != hi[3]:
                rng = hi[3] - lo[3]
                dd = vias[el[j]][i][3] - nm[3]
                while dd > 0.5 * rng:
                    dd -= rng
                while dd < -0.5 * rng:
                    dd += rng
                diff[3] = dd
            for d in range(4):
                ve[d] += w[j] * (diff[d] * diff[d])
        for d in range(4):
            blend = (1.0 - var_beta) * (sigma[i][d] * sigma[i][d]) + var_beta * ve[d]
            sigma[i][d] = clampsd(clampsd(math.sqrt(blend)) * dec)
    return sigma, mean, el[0], el


def random_list(seed, n, K, p_succ=0.5, ties=False):
    rng = np.random.default_rng(seed)
    vias = rng.uniform(-1.5, 1.5, (n, K, 4))
    cost = rng.uniform(0.0, 3.0, n)
    if ties:
        cost = np.round(cost, 1)
    status = (rng.uniform(size=n) < p_succ).astype(np.uint8)
    return cost, status, vias


@pytest.mark.parametrize("seed,n,K,ties", [(0, 52, 1, False), (1, 300, 2, True), (2, 7, 3, False),
                                           (3, 1000, 1, True), (4, 130, 4, False)])
def test_oracle_update_matches_literal_reference(seed, n, K, ties):
    cost, status, vias = random_list(seed, n, K, ties=ties)
    m0, s0 = O.ces_reset([0, 0, 0.1, 0], [1, -1, 0.5, 1.2], K + 2)
    lit_s, lit_m, lit_best, lit_el = literal_update(cost, status, vias, m0, s0)
    for seq in (True, False):
        m, s, lb, hb, ns, el, bs = O.ces_update(cost, status, vias, m0, s0, np.zeros((K, 4)), False,
                                                sequential=seq)
        assert ns == int(status.sum()) and hb
        assert list(el) == lit_el and bs == lit_best
        np.testing.assert_array_equal(lb, vias[lit_best])
        if seq:  # reference summation order: bit-identical
            np.testing.assert_array_equal(m, np.array(lit_m))
            np.testing.assert_array_equal(s, np.array(lit_s))
        else:    # canonical wave order (the GPU's): within rounding
            assert np.abs(m - np.array(lit_m)).max() <= 1e-12
            assert np.abs(s - np.array(lit_s)).max() <= 1e-12


def test_oracle_update_no_success_and_limits():
    K = 2
    cost, status, vias = random_list(5, 40, K, p_succ=0.0)
    m0 = np.full((K, 4), 0.1)
    s0 = np.array([[0.3, 0.49, 0.009, 0.2]] * K)
    m, s, lb, hb, ns, el, bs = O.ces_update(cost, status, vias, m0, s0, np.zeros((K, 4)), False)
    assert ns == 0 and not hb and bs == -1 and len(el) == 0
    np.testing.assert_array_equal(m, m0)  # mean untouched, sigma *= inc then clamped
    np.testing.assert_array_equal(s, np.clip(s0 * 1.5, 0.01, 0.5))


def test_reset_reproduces_q1_z_clamp():
    # TaskSpacePlanner hands stddev_initial to Planner's z_min (tsp.h:53): the mean's z is
    # clamped to >= stddev_initial (0.3) even though cfg.z_min is 0
    m, s = O.ces_reset([0.2, 0, 0.1, 0], [0, 0, 0.12, 0], 3)
    assert m[0, 2] == 0.3 and m[0, 0] == 0.1 and (s == 0.3).all()
    m, s = O.ces_reset([0.2, 0, 0.1, 0], [0, 0, 0.12, 0], 3, dist_z_min=0.0, sd_max=0.2)
    assert m[0, 2] == 0.5 * 0.1 + 0.5 * 0.12 and (s == 0.2).all()


def test_yaw_wrap_in_variance():
    # elites straddling the +-pi seam: wrapped differences keep the yaw variance small
    K = 1
    vias = np.zeros((4, K, 4))
    vias[:, 0, 3] = [3.1, -3.1, 3.05, -3.05]
    cost = np.array([1.0, 1.1, 1.2, 1.3])
    st = np.ones(4, np.uint8)
    m0 = np.array([[0, 0, 0.5, 3.1]])
    s0 = np.full((K, 4), 0.3)
    lo, hi = (-2.0, -2.0, 0.0, -math.pi), (2.0, 2.0, 2.0, math.pi)
    m, s, *_ = O.ces_update(cost, st, vias, m0, s0, np.zeros((K, 4)), False, frac=1.0, lo=lo, hi=hi)
    lit_s, lit_m, _, _ = literal_update(cost, st, vias, m0, s0, frac=1.0, lo=lo, hi=hi)
    assert np.abs(s - np.array(lit_s)).max() <= 1e-12
    assert np.abs(m - np.array(lit_m)).max() <= 1e-12


def test_oracle_plan_loop_forwards_best():
    import sspp_amd as S
    osc = O.Scene(mjcf_ref.load(STACKING), 1, S.Model(STACKING).body_id("block1"))
    start, end = np.array([0.205, 0.0, 0.12, 0.0]), np.array([0.0, 0.0, 0.32, 0.0])
    recs = O.ces_plan(osc, start, end, iterations=3, samples=60, checks=40, lo=LO, hi=HI)
    for t, r in enumerate(recs):
        assert len(r["vias"]) == 60 + (2 if t > 0 and recs[t - 1]["has_best"] else 1)
        if t > 0 and recs[t - 1]["has_best"]:
            np.testing.assert_array_equal(r["vias"][1], recs[t - 1]["last_best"])
    assert any(r["n_success"] > 0 for r in recs)


# ------------------------------------------------------------------ device planner
def stacking_planner(samples, checks=64, init_points=3, seed=0x5EED, world=1, rank=0, **kw):
    import sspp_amd as S
    model = S.Model(STACKING)
    scene = S.Scene(model, 1, model.body_id("block1"))
    pl = S.CesPlanner(scene, sample_count=samples, check_points=checks, init_points=init_points,
                      limits_min=LO, limits_max=HI, seed=seed, world=world, rank=rank, **kw)
    osc = O.Scene(mjcf_ref.load(STACKING), 1, model.body_id("block1"))
    start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
    end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
    return pl, scene, osc, start, end


@pytest.mark.gpu
@pytest.mark.parametrize("samples,checks,init_points", [(50, 50, 3), (2000, 128, 3), (333, 40, 5),
                                                        (16384, 128, 3)])
def test_device_ces_matches_oracle_each_iteration(cuda, samples, checks, init_points):
    pl, scene, osc, start, end = stacking_planner(samples, checks, init_points)
    K = init_points - 2
    prev = None
    seen_success = seen_forward = False
    for t in range(6):
        if prev is None:
            m_in, s_in = O.ces_reset(start, end, init_points, lo=LO, hi=HI)
            lb_in, hb_in = np.zeros((K, 4)), False
        else:
            m_in, s_in, lb_in, hb_in = prev["mean"], prev["sigma"], prev["last_best"], prev["has_best"]
        pl.step(start, end, iterate=t > 0)
        r = pl.read()
        # seed list: mean set (z >= cfg.z_min = 0), forwarded best, then Philox samples
        nfx = 2 if (t > 0 and hb_in) else 1
        assert r["n_fixed"] == nfx and r["n_candidates"] == nfx + samples
        np.testing.assert_array_equal(r["vias"][0], np.where(np.arange(4) == 2, np.maximum(m_in, 0.0), m_in))
        if nfx == 2:
            np.testing.assert_array_equal(r["vias"][1], lb_in)
            seen_forward = True
        smp = O.sample_tsp(m_in, s_in, LO, HI, 0.0, 0x5EED, t * samples, samples)
        assert np.abs(r["vias"][nfx:] - smp).max() <= 1e-12
        # per-candidate costs vs the oracle on the device's own via sets
        L, Cnf, Cwf, st, cost = O.tsp_score(osc, start, end, r["vias"], checks)
        np.testing.assert_array_equal(r["status"], st)
        for a, b in ((r["L"], L), (r["C_nf"], Cnf), (r["C_wf"], Cwf), (r["cost"], cost)):
            assert np.abs(a - b).max() <= 1e-9
        # the update on the device's results: identical elites/best, bit-identical distribution
        m, s, lb, hb, ns, el, bs = O.ces_update(r["cost"], r["status"], r["vias"], m_in, s_in,
                                                lb_in, hb_in, lo=LO, hi=HI)
        assert r["n_success"] == ns and r["best_slot"] == bs and r["has_best"] == hb
        np.testing.assert_array_equal(r["elites"], el)
        np.testing.assert_array_equal(r["mean"], m)
        np.testing.assert_array_equal(r["sigma"], s)
        np.testing.assert_array_equal(r["last_best"], lb)
        seen_success |= ns > 0
        prev = r
    assert seen_success
    if samples >= 2000:
        assert seen_forward


@pytest.mark.gpu
def test_device_plan_iterations_equals_stepping(cuda):
    a, _, _, start, end = stacking_planner(500)
    b, _, _, _, _ = stacking_planner(500)
    a.plan(start, end, iterate=False, iterations=8)
    for t in range(8):
        b.step(start, end, iterate=t > 0)
    ra, rb = a.read(), b.read()
    for k in ("mean", "sigma", "last_best", "cost", "status", "vias", "elites"):
        np.testing.assert_array_equal(ra[k], rb[k])
    assert ra["iteration"] == rb["iteration"] == 8


@pytest.mark.gpu
def test_read_after_operations_on_several_streams(cuda):
    """begin / eval / update each on its own (then destroyed) stream: read() still returns the
    finished iteration (it waits on the whole device when the planner's operations since the
    previous read used more than one stream), equal to the same iteration on one stream."""
    import torch
    a, _, _, start, end = stacking_planner(2000)
    b, _, _, _, _ = stacking_planner(2000)
    for t in range(3):
        s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        a.begin(start, end, t > 0, stream=s1)
        s2.wait_stream(s1)
        a.eval(stream=s2)
        s3.wait_stream(s2)
        a.update(stream=s3)
        del s1, s2, s3
        ra = a.read()
        b.step(start, end, iterate=t > 0)
        rb = b.read()
        for k in ("mean", "sigma", "last_best", "cost", "status", "vias", "elites"):
            np.testing.assert_array_equal(ra[k], rb[k], err_msg="%s at %d" % (k, t))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_multirank_exchange_equals_single_rank(cuda, world):
    """world ranks emulated in one process: each evaluates its slots, the packed records are
    concatenated (what all_gather_into_tensor does) and unpacked on every rank; every rank's
    update must equal the single-rank planner's."""
    import ctypes as C
    import torch
    from sspp_amd._lib import lib
    from sspp_amd.runtime import _ptr, _stream
    samples = 777
    ref, _, _, start, end = stacking_planner(samples)
    ranks = [stacking_planner(samples, world=world, rank=r)[0] for r in range(world)]
    rec = 5 + 4 * ranks[0].K
    for t in range(5):
        ref.step(start, end, iterate=t > 0)
        parts = []
        for r, pl in enumerate(ranks):
            pl.begin(start, end, t > 0)
            pl.eval()
            buf = torch.empty(pl.spr * rec, dtype=torch.float64, device="cuda")
            assert lib().sspp_ces_pack(pl._h, r, _ptr(buf), _stream(None)) == 0
            parts.append(buf)
        full = torch.cat(parts)
        for pl in ranks:
            assert lib().sspp_ces_unpack(pl._h, _ptr(full), _stream(None)) == 0
            pl.update()
        want = ref.read()
        for pl in ranks:
            got = pl.read()
            for k in ("mean", "sigma", "last_best", "elites", "cost", "status", "vias"):
                np.testing.assert_array_equal(got[k], want[k])
            assert got["best_slot"] == want["best_slot"]
    del C


@pytest.mark.gpu
def test_tsp_module_surface(cuda):
    import sys
    from sspp import _tsp
    p = _tsp.TaskSpacePlanner(STACKING, "block1", sample_count=400, check_points=64,
                              limits_min=np.array(LO), limits_max=np.array(HI))
    start = np.array([0.205, 0.0, 0.12, 0.0])
    end = np.array([0.0, 0.0, 0.32, 0.0])
    succ = p.plan(start, end, False)
    assert all(c.status == _tsp.SolverStatus.Converged and c.C_nf == 0.0 for c in succ)
    fail = p.get_failed_path_candidates()
    assert len(succ) + len(fail) == 401 == len(p.get_sampled_via_sets())
    assert all(c.status == _tsp.SolverStatus.Failed for c in fail)
    vp = p.get_via_pts()
    assert len(vp) == 3 and np.allclose(vp[0], start) and np.allclose(vp[2], end)
    it = [p.plan(start, end, True) for _ in range(4)]
    assert len(p.get_sampled_via_sets()) == 402  # mean set + forwarded best + samples
    best = min(it[-1], key=lambda c: c.L + 1.0 * c.C_wf) if it[-1] else None
    if best is not None:
        s = p.spline_from_vias(best.via)
        np.testing.assert_allclose(p.evaluate(0.37), s(0.37), rtol=0, atol=1e-15)
        np.testing.assert_allclose(p.get_ctrl_pts(), s.ctrls(), rtol=0, atol=0)
    pts = p.get_path_pts(5)
    assert len(pts) == 5 and np.allclose(pts[0], start, atol=1e-12) and np.allclose(pts[-1], end, atol=1e-12)
    assert p.get_knot_vector().shape == (6,)
    assert p.get_current_stddev().shape == (4,)
    with pytest.raises(RuntimeError):
        _tsp.TaskSpacePlanner(STACKING, "no_such_body")
    assert _tsp.__backend__ == "hip-gfx950" and "sspp._tsp" in sys.modules


@pytest.mark.gpu
def test_config5_multigoal_full_size_each_iteration(cuda):
    """BASELINE configs[4] at its stated size: the gripper TaskSpacePlanner (7 collidable geoms)
    on robocrane.xml, 4096 sampled via sets x 128 checks, all 8 bench goals, 3 CES iterations
    each (tsp_planner.h:72-145).  Per iteration, against the oracle on the device's own via sets:
    status identical, costs <= 1e-9, then elites / best slot / mean / sigma bit-identical."""
    import bench
    import sspp_amd as S
    model = S.Model(ROBOCRANE)
    body = model.body_id("gripper_collision_with_block/")
    scene = S.Scene(model, 1, body)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 1, body)
    lo, hi = bench.MG_LO, bench.MG_HI
    samples, checks = 4096, 128
    seen_success = 0
    for g, (st, en) in enumerate(bench.MULTIGOAL):
        st, en = np.array(st), np.array(en)
        pl = S.CesPlanner(scene, sample_count=samples, check_points=checks, init_points=3,
                          limits_min=lo, limits_max=hi, seed=S.DEFAULT_SEED + g)
        prev = None
        for t in range(3):
            if prev is None:
                m_in, s_in = O.ces_reset(st, en, 3, lo=lo, hi=hi)
                lb_in, hb_in = np.zeros((1, 4)), False
            else:
                m_in, s_in, lb_in, hb_in = prev["mean"], prev["sigma"], prev["last_best"], prev["has_best"]
            pl.step(st, en, iterate=t > 0)
            r = pl.read()
            nfx = 2 if (t > 0 and hb_in) else 1
            assert r["n_fixed"] == nfx and r["n_candidates"] == nfx + samples
            smp = O.sample_tsp(m_in, s_in, lo, hi, 0.0, S.DEFAULT_SEED + g, t * samples, samples)
            assert np.abs(r["vias"][nfx:] - smp).max() <= 1e-12
            L, Cnf, Cwf, stt, cost = O.tsp_score(osc, st, en, r["vias"], checks)
            np.testing.assert_array_equal(r["status"], stt)
            fin = np.isfinite(cost)
            np.testing.assert_array_equal(np.isfinite(r["cost"]), fin)
            # relative 1e-12: colliding gripper candidates sum hundreds of contact terms, and the
            # device's control points come from the collocation inverse, not a per-candidate QR
            for a, b in ((r["cost"][fin], cost[fin]), (r["L"], L), (r["C_nf"], Cnf), (r["C_wf"], Cwf)):
                assert (np.abs(a - b) <= 1e-12 * np.maximum(1.0, np.abs(b))).all()
            m, s, lb, hb, ns, el, bs = O.ces_update(r["cost"], r["status"], r["vias"], m_in, s_in,
                                                    lb_in, hb_in, lo=lo, hi=hi)
            assert r["n_success"] == ns and r["best_slot"] == bs and r["has_best"] == hb
            np.testing.assert_array_equal(r["elites"], el)
            np.testing.assert_array_equal(r["mean"], m)
            np.testing.assert_array_equal(r["sigma"], s)
            np.testing.assert_array_equal(r["last_best"], lb)
            seen_success += ns > 0
            prev = r
    assert seen_success >= 8  # most goals find collision-free via sets


@pytest.mark.gpu
@pytest.mark.parametrize("unfused", [0, 1])
def test_icra_anytime_size_each_iteration(cuda, unfused):
    """The reference's ICRA anytime configuration (src/main_icra_benchmark.cpp:151-179: 15
    samples x 40 checks, 1 via, gripper on robocrane.xml, block_green -> block_orange): 20
    iterations, each against the oracle.  17 slots take the one-launch update (ranking inside
    k_ces_update); the SSPP_OPT_CES_FUSED = 0 option forces rank + scatter + update — both
    bit-identical."""
    import bench
    import sspp_amd as S
    cfg = bench.ICRA
    model = S.Model(ROBOCRANE)
    body = model.body_id(bench.ICRA_BODY)
    scene = S.Scene(model, 1, body)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 1, body)
    lo, hi = cfg["limits_min"], cfg["limits_max"]
    st = model.body_point("block_green/") + np.array([0, 0, 0.02, 0])
    en = model.body_point("block_orange/") + np.array([0, 0, 0.02, 0])
    kw = {k: cfg[k] for k in ("stddev_initial", "stddev_min", "stddev_max", "stddev_increase_factor",
                              "stddev_decay_factor", "elite_fraction", "sample_count", "check_points",
                              "init_points", "collision_weight", "z_min", "sigma_floor", "var_ema_beta",
                              "mean_lr")}
    pl = S.CesPlanner(scene, limits_min=lo, limits_max=hi, **kw)
    if unfused:
        pl.set_option(S.OPT_CES_FUSED, 0)
    ocfg = dict(frac=cfg["elite_fraction"], inc=cfg["stddev_increase_factor"],
                dec=cfg["stddev_decay_factor"], sigma_floor=cfg["sigma_floor"], var_beta=cfg["var_ema_beta"],
                mean_lr=cfg["mean_lr"], sd_min=cfg["stddev_min"], sd_max=cfg["stddev_max"],
                dist_z_min=cfg["stddev_initial"], lo=lo, hi=hi)
    samples, z_min = cfg["sample_count"], cfg["z_min"]
    m_in, s_in = O.ces_reset(st, en, 3, z_min, cfg["stddev_initial"], 0.3, cfg["stddev_min"],
                             cfg["stddev_max"], cfg["sigma_floor"], lo, hi)
    lb_in, hb_in = np.zeros((1, 4)), False
    succ = 0
    for t in range(20):
        pl.step(st, en, iterate=t > 0)
        r = pl.read()
        nfx = 2 if (t > 0 and hb_in) else 1
        assert r["n_fixed"] == nfx and r["n_candidates"] == nfx + samples
        np.testing.assert_array_equal(r["vias"][0], np.where(np.arange(4) == 2, np.maximum(m_in, z_min), m_in))
        smp = O.sample_tsp(m_in, s_in, lo, hi, z_min, S.DEFAULT_SEED, t * samples, samples)
        assert np.abs(r["vias"][nfx:] - smp).max() <= 1e-12
        L, Cnf, Cwf, stt, cost = O.tsp_score(osc, st, en, r["vias"], cfg["check_points"])
        np.testing.assert_array_equal(r["status"], stt)
        fin = np.isfinite(cost)
        for a, b in ((r["cost"][fin], cost[fin]), (r["L"], L), (r["C_nf"], Cnf), (r["C_wf"], Cwf)):
            assert (np.abs(a - b) <= 1e-12 * np.maximum(1.0, np.abs(b))).all()
        m, s, lb, hb, ns, el, bs = O.ces_update(r["cost"], r["status"], r["vias"], m_in, s_in, lb_in, hb_in,
                                                **ocfg)
        assert r["n_success"] == ns and r["best_slot"] == bs and r["has_best"] == hb
        np.testing.assert_array_equal(r["elites"], el)
        np.testing.assert_array_equal(r["mean"], m)
        np.testing.assert_array_equal(r["sigma"], s)
        np.testing.assert_array_equal(r["last_best"], lb)
        succ += ns > 0
        m_in, s_in, lb_in, hb_in = m, s, lb, hb
    assert succ >= 10


@pytest.mark.gpu
def test_elite_fraction_above_one_rejected(cuda):
    """tsp_elites.h:15-19 would partial_sort past the end for frac > 1: rejected at creation."""
    import sspp_amd as S
    model = S.Model(STACKING)
    scene = S.Scene(model, 1, model.body_id("block1"))
    with pytest.raises(S.SsppError, match="elite_fraction"):
        S.CesPlanner(scene, sample_count=100, check_points=32, elite_fraction=1.5)
    S.CesPlanner(scene, sample_count=100, check_points=32, elite_fraction=1.0)  # accepted


@pytest.mark.gpu
@pytest.mark.parametrize("samples,iters", [(4096, 3), (300, 2)])
def test_ces_plan_group_matches_single(cuda, samples, iters):
    """sspp_ces_plan_group (BASELINE configs[4]: every goal's CES iteration in one chain of batched
    launches, one k_tsp_group evaluation per iteration) against each planner's own sspp_ces_plan:
    every read() field bit-identical per goal after `iters` iterations, then one more iteration
    continuing both (iterate=True).  300 samples is the pair-split size: the group runs goal by
    goal there, with the same results."""
    import bench
    import sspp_amd as S
    model = S.Model(ROBOCRANE)
    body = model.body_id("gripper_collision_with_block/")
    scene = S.Scene(model, 1, body)
    goals = bench.MULTIGOAL
    starts = np.array([g[0] for g in goals])
    ends = np.array([g[1] for g in goals])

    def make():
        return [S.CesPlanner(scene, sample_count=samples, check_points=128, init_points=3,
                             limits_min=bench.MG_LO, limits_max=bench.MG_HI, seed=S.DEFAULT_SEED + g)
                for g in range(len(goals))]
    solo, group = make(), make()
    for p, st, en in zip(solo, starts, ends):
        p.plan(st, en, iterate=False, iterations=iters)
    S.CesPlanner.plan_group(group, starts, ends, iterate=False, iterations=iters)
    for round_ in range(2):
        for g, (a, b) in enumerate(zip(solo, group)):
            ra, rb = a.read(), b.read()
            for k in ra:
                np.testing.assert_array_equal(np.asarray(ra[k]), np.asarray(rb[k]), err_msg="goal %d %s" % (g, k))
        if round_ == 0:
            for p, st, en in zip(solo, starts, ends):
                p.plan(st, en, iterate=True, iterations=1)
            S.CesPlanner.plan_group(group, starts, ends, iterate=True, iterations=1)
    assert sum(p.read()["n_success"] for p in solo) > 0


@pytest.mark.gpu
def test_ces_plan_group_matches_oracle(cuda):
    """k_tsp_group (the multi-goal bench's evaluation: every goal's slots in one grid) directly
    against the oracle, not through the per-goal planners: BASELINE configs[4] at 4096 samples x
    128 checks, all 8 goals, two group iterations (reset, then iterate with the forwarded best).
    Per goal and iteration, on the device's own via sets: the Philox samples, status, costs
    (<= 1e-12 relative), then elites / best slot / mean / sigma / last best bit-identical to
    O.ces_update (tsp_planner.h:121-142)."""
    import bench
    import sspp_amd as S
    model = S.Model(ROBOCRANE)
    body = model.body_id("gripper_collision_with_block/")
    scene = S.Scene(model, 1, body)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 1, body)
    lo, hi = bench.MG_LO, bench.MG_HI
    samples, checks = 4096, 128
    goals = bench.MULTIGOAL
    starts = np.array([g[0] for g in goals])
    ends = np.array([g[1] for g in goals])
    pls = [S.CesPlanner(scene, sample_count=samples, check_points=checks, init_points=3, limits_min=lo,
                        limits_max=hi, seed=S.DEFAULT_SEED + g) for g in range(len(goals))]
    prev = [None] * len(goals)
    for t in range(2):
        S.CesPlanner.plan_group(pls, starts, ends, iterate=t > 0, iterations=1)
        for g, pl in enumerate(pls):
            st, en = starts[g], ends[g]
            if prev[g] is None:
                m_in, s_in = O.ces_reset(st, en, 3, lo=lo, hi=hi)
                lb_in, hb_in = np.zeros((1, 4)), False
            else:
                p = prev[g]
                m_in, s_in, lb_in, hb_in = p["mean"], p["sigma"], p["last_best"], p["has_best"]
            r = pl.read()
            nfx = 2 if (t > 0 and hb_in) else 1
            assert r["n_fixed"] == nfx and r["n_candidates"] == nfx + samples
            smp = O.sample_tsp(m_in, s_in, lo, hi, 0.0, S.DEFAULT_SEED + g, t * samples, samples)
            assert np.abs(r["vias"][nfx:] - smp).max() <= 1e-12
            L, Cnf, Cwf, stt, cost = O.tsp_score(osc, st, en, r["vias"], checks)
            np.testing.assert_array_equal(r["status"], stt)
            fin = np.isfinite(cost)
            np.testing.assert_array_equal(np.isfinite(r["cost"]), fin)
            for a, b in ((r["cost"][fin], cost[fin]), (r["L"], L), (r["C_nf"], Cnf), (r["C_wf"], Cwf)):
                assert (np.abs(a - b) <= 1e-12 * np.maximum(1.0, np.abs(b))).all()
            m, s, lb, hb, ns, el, bs = O.ces_update(r["cost"], r["status"], r["vias"], m_in, s_in, lb_in, hb_in,
                                                    lo=lo, hi=hi)
            assert r["n_success"] == ns and r["best_slot"] == bs and r["has_best"] == hb
            np.testing.assert_array_equal(r["elites"], el)
            np.testing.assert_array_equal(r["mean"], m)
            np.testing.assert_array_equal(r["sigma"], s)
            np.testing.assert_array_equal(r["last_best"], lb)
            prev[g] = r
    assert sum(p["n_success"] > 0 for p in prev) >= 6

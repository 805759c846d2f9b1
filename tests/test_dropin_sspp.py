"""The drop-in `from sspp import _sspp` surface (src/sspp_bindings.cpp:14-69) on the GPU."""
import os

import numpy as np
import pytest

from oracle import mjcf_ref
from oracle import oracle as O
from tests.conftest import SCENES

pytestmark = pytest.mark.gpu
ROBOCRANE = os.path.join(SCENES, "robocrane.xml")


@pytest.fixture(scope="module")
def sp(cuda):
    from sspp import _sspp
    assert _sspp.__backend__ == "hip-gfx950"
    return _sspp


def test_plan_matches_oracle(sp, capfd):
    planner = sp.SamplingPathPlanner7(ROBOCRANE)
    start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707]).reshape(7, 1)  # (N,1) accepted
    sigma, limits = 0.1, np.ones((7, 1))
    ok, paths = planner.plan(start, end, sigma, limits, sample_count=512, check_points=64,
                             init_points=10)
    out = capfd.readouterr().out
    assert "Sampled 512 splines. Successful paths found: %d" % len(paths) in out
    # oracle on the same candidates
    init = sp.Spline7()
    assert planner.initializePath(start, end, init, 10)
    knots = init.knots()
    ctrl0 = init.ctrls().T.copy()
    ctrl = O.sample_sspp(ctrl0, 3, sigma, np.ones(7), planner.seed, 0, 512)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7)
    arc, feas = O.sspp_score(osc, knots, 3, ctrl, 64)
    assert len(paths) == int(feas.sum())
    assert ok == (feas.sum() > 0)
    feas_idx = np.nonzero(feas)[0]
    for s, i in zip(paths, feas_idx):
        np.testing.assert_allclose(s.ctrls().T, ctrl[i], rtol=0, atol=1e-12)
    if ok:
        idx, best = O.argmin(arc, feas)
        assert planner.last_best_index == idx
        np.testing.assert_allclose(planner.get_ctrl_pts().T, ctrl[idx], atol=1e-12)
        np.testing.assert_allclose(planner.evaluate(0.0), start, atol=1e-12)
        np.testing.assert_allclose(planner.evaluate(1.0), end.ravel(), atol=1e-12)
        # computeArcLength / findBestPath agree with plan's internal argmin
        assert abs(planner.computeArcLength(paths[0], 64) - arc[feas_idx[0]]) <= 1e-12
        bs = sp.Spline7()
        assert planner.findBestPath(paths, bs, 64)
        np.testing.assert_allclose(bs.ctrls(), planner.get_ctrl_pts(), atol=0)


def test_spline_views_and_helpers(sp):
    planner = sp.SamplingPathPlanner7(ROBOCRANE)
    s = sp.Spline7()
    assert s.ctrls().shape == (7, 0)
    start = np.zeros(7) + [0.3, 0.2, 0.5, 1, 0, 0, 0]
    end = start + [0.2, 0, 0, 0, 0, 0, 0]
    planner.initializePath(start, end, s, 7)
    c = s.ctrls()
    assert c.shape == (7, 7)
    c[0, 3] += 0.5  # view semantics (reference_internal)
    assert s.ctrls()[0, 3] == c[0, 3]
    noisy = planner.sampleWithNoise(s, 0.1, np.ones(7), 3)
    assert noisy.ctrls().shape == (7, 7)
    np.testing.assert_array_equal(noisy.ctrls()[:, :3], s.ctrls()[:, :3])  # j < p fixed
    assert not planner.checkCollision(s, 20)  # hovering at z=0.5, far from everything
    low = sp.Spline7()
    planner.initializePath(start - [0, 0, 0.49, 0, 0, 0, 0], end - [0, 0, 0.49, 0, 0, 0, 0], low, 7)
    assert planner.checkCollision(low, 20)  # through the floor
    with pytest.raises(TypeError):
        planner.sampleWithNoise(s, 0.1, np.ones(7), object())
    with pytest.raises(ValueError):
        planner.plan(np.zeros(6), np.zeros(7), 0.1, np.ones(7))


def test_bad_path_raises(sp):
    with pytest.raises(RuntimeError):
        sp.SamplingPathPlanner7("/nonexistent/scene.xml")


def test_other_dofs(sp):
    """SamplingPathPlanner3/6/9 on the same scene (qpos window semantics, include/sspp.h:139-142)."""
    for cls, N in ((sp.SamplingPathPlanner3, 3), (sp.SamplingPathPlanner6, 6),
                   (sp.SamplingPathPlanner9, 9)):
        planner = cls(ROBOCRANE)
        q0 = np.array([0.5, 0.15, 0.3, 0.707, 0, 0, 0.707, 0.5, -0.05])[:N]
        q1 = q0.copy()
        q1[1] = -0.05
        ok, paths = planner.plan(q0, q1, 0.02, np.ones(N), sample_count=64, check_points=32,
                                 init_points=6)
        osc = O.Scene(mjcf_ref.load(ROBOCRANE), 0, N)
        init = getattr(sp, "Spline%d" % N)()
        planner.initializePath(q0, q1, init, 6)
        ctrl = O.sample_sspp(init.ctrls().T.copy(), 3, 0.02, np.ones(N), planner.seed, 0, 64)
        arc, feas = O.sspp_score(osc, init.knots(), 3, ctrl, 32)
        assert len(paths) == int(feas.sum())
        assert ok == bool(feas.any())


def test_evaluate_returns_ndarray(sp):
    """Eigen Matrix<double, N, 1> returns reach Python as numpy arrays of shape (N,)."""
    planner = sp.SamplingPathPlanner7(ROBOCRANE)
    s = sp.Spline7()
    start = np.array([0.3, 0.2, 0.5, 1, 0, 0, 0])
    planner.initializePath(start, start + [0.2, 0, 0, 0, 0, 0, 0], s, 7)
    for v in (planner.evaluate(s, 0.5), s(0.5)):
        assert isinstance(v, np.ndarray) and v.shape == (7,) and v.dtype == np.float64
    np.testing.assert_allclose(planner.evaluate(s, 0.0) - start, np.zeros(7), atol=1e-12)


def test_check_collision_one_sample(sp):
    """include/sspp.h:132-150 with num_samples = 1 checks only u = 0 and u = 1."""
    planner = sp.SamplingPathPlanner7(ROBOCRANE)
    start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])  # the straight line crosses the bricks
    s = sp.Spline7()
    planner.initializePath(start, end, s, 10)
    assert not planner.checkCollision(s, 1)   # both end points are free
    assert planner.checkCollision(s, 20)      # the middle is not


def test_plan_cached_state_across_shapes(sp, capfd):
    """The cached device planner (sspp_planner_plan) re-targets its job between calls: every
    call must still equal the oracle, whatever the shape sequence (same shape, new start/end,
    new sigma, larger and smaller batches, other init_points / check_points)."""
    planner = sp.SamplingPathPlanner7(ROBOCRANE)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7)
    base_s = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    base_e = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
    calls = [(base_s, base_e, 0.08, 1024, 64, 10), (base_s, base_e, 0.08, 1024, 64, 10),
             (base_s + [0, 0, 0.05, 0, 0, 0, 0], base_e, 0.12, 1024, 64, 10),
             (base_s, base_e, 0.08, 3000, 64, 10), (base_s, base_e, 0.05, 700, 64, 10),
             (base_s, base_e, 0.08, 512, 96, 8), (base_s, base_e, 0.08, 512, 96, 8)]
    for k, (st, en, sig, B, W, n) in enumerate(calls):
        planner.seed = 1000 + k
        ok, paths = planner.plan(st, en, sig, np.ones(7), sample_count=B, check_points=W, init_points=n)
        init = sp.Spline7()
        planner.initializePath(st, en, init, n)
        ctrl = O.sample_sspp(init.ctrls().T.copy(), 3, sig, np.ones(7), planner.seed, 0, B)
        arc, feas = O.sspp_score(osc, init.knots(), 3, ctrl, W)
        ids = np.nonzero(feas)[0]
        assert list(planner.last_feasible_ids) == list(ids)
        assert len(paths) == len(ids) and ok == bool(len(ids))
        for s, i in zip(paths, ids):
            np.testing.assert_allclose(s.ctrls().T, ctrl[i], rtol=0, atol=1e-12)
        if ok:
            idx, best = O.argmin(arc, feas)
            assert planner.last_best_index == idx
            assert abs(planner.last_best_cost - best) <= 1e-12
            np.testing.assert_allclose(planner.get_ctrl_pts().T, ctrl[idx], atol=1e-12)
    capfd.readouterr()


def test_plan_sspp_c_abi_cached(cuda):
    """sspp_plan_sspp (the blocking all-candidates plan() of the C ABI) on
    its cached planner: repeated calls, a shape change and a freed-and-recreated scene, each
    against the oracle on the same Philox candidates."""
    import ctypes as C
    import sspp_amd as S
    from sspp_amd._lib import Best, lib
    L = lib()
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7)
    start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
    lim = np.ones(7)
    p = lambda a, t=C.c_double: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    nfeas = 0
    for round_ in range(2):
        scene = S.Scene(S.Model(ROBOCRANE), 0, 7)
        for B, W, n, seed in ((2000, 64, 10, 7), (2000, 64, 10, 8), (777, 48, 6, 9), (1500, 64, 10, 10)):
            knots, ctrl = np.zeros(n + 4), np.zeros((B, n, 7))
            feas, arc, best = np.zeros(B, np.uint8), np.zeros(B), Best()
            rc = L.sspp_plan_sspp(scene.handle, 7, p(start), p(end), C.c_double(0.08), p(lim), B, W, n,
                                  C.c_uint64(seed), p(knots), p(ctrl), p(feas, C.c_uint8), p(arc), C.byref(best))
            assert rc == 0, L.sspp_last_error()
            u = np.array([i / (n - 1) for i in range(n)])
            k0, c0 = O.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
            np.testing.assert_allclose(knots, k0, rtol=0, atol=1e-15)
            want = O.sample_sspp(c0, 3, 0.08, lim, seed, 0, B)
            assert np.abs(ctrl - want).max() <= 1e-12
            oarc, ofeas = O.sspp_score(osc, knots, 3, ctrl, W)
            np.testing.assert_array_equal(feas, ofeas)
            fin = ofeas.astype(bool)
            nfeas += int(fin.sum())
            if fin.any():
                assert np.abs(arc[fin] - oarc[fin]).max() <= 1e-12
                assert best.index == O.argmin(oarc, ofeas)[0]
            else:
                assert best.index == -1
        del scene  # sspp_scene_free drops the cached planner of this scene
    assert nfeas > 0


def test_static_contacts_count_like_the_reference(sp):
    """checkCollision's ncon is the whole scene's (include/sspp.h:143-144): in
    stacking.xml block2 and block3 rest on the floor (MuJoCo's plane-box collider counts a
    corner at distance 0), so every candidate of a planner moving block1 is in collision, as in
    the reference; the robocrane scene has no static contact, so its results do not change."""
    stacking = os.path.join(SCENES, "stacking.xml")
    osc = O.Scene(mjcf_ref.load(stacking), 0, 7)
    q = np.array([0.2, 0.0, 0.4, 1.0, 0.0, 0.0, 0.0])  # block1 lifted clear of everything
    assert osc.contacts(q)[0] == 0 and osc.contacts(q, count_static=True)[0] == 8
    planner = sp.SamplingPathPlanner7(stacking)
    start = q
    end = np.array([0.0, 0.2, 0.4, 1.0, 0.0, 0.0, 0.0])
    ok, paths = planner.plan(start, end, 0.01, np.ones(7), sample_count=256, check_points=32,
                             init_points=10)
    assert not ok and len(paths) == 0
    init = sp.Spline7()
    assert planner.initializePath(start, end, init, 10)
    arc, feas = O.sspp_score(osc, init.knots(), 3, init.ctrls().T.copy()[None], 32, count_static=True)
    assert not feas.any()


def _planner_plan(L, pl, start, end, sigma, B, W, n, seed):
    """sspp_planner_plan through the C ABI: (feasible ids, their arcs, their control points, best)."""
    import ctypes as C
    from sspp_amd import _lib
    d = C.POINTER(C.c_double)
    st, en, lim = (np.ascontiguousarray(x, dtype=np.float64) for x in (start, end, np.ones(7)))
    knots = np.zeros(n + 4)
    nf = C.c_int64()
    ids = np.zeros(B, dtype=np.int64)
    arcs = np.zeros(B)
    ctrl = np.zeros((B, n, 7))
    best = _lib.Best()
    _lib.check(L.sspp_planner_plan(pl, st.ctypes.data_as(d), en.ctypes.data_as(d), sigma, lim.ctypes.data_as(d),
                                   B, W, n, seed, 0, knots.ctypes.data_as(d), C.byref(nf),
                                   ids.ctypes.data_as(C.POINTER(C.c_int64)), arcs.ctypes.data_as(d),
                                   ctrl.ctypes.data_as(d), C.byref(best)), "sspp_planner_plan")
    k = nf.value
    return ids[:k], arcs[:k], ctrl[:k], knots, (best.cost, best.index, best.count)


def _prepass_state(L, pl):
    import ctypes as C
    from sspp_amd import _lib
    v = C.c_int64()
    _lib.check(L.sspp_planner_get_option(pl, _lib.OPT_PREPASS_STATE, C.byref(v)), "get_option")
    return v.value


def _check_plan(osc, res, start, end, sigma, B, W, n, seed):
    import sspp_amd as S
    ids, arcs, ctrl, knots, best = res
    u = np.array([i / (n - 1) for i in range(n)])
    k2, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
    np.testing.assert_array_equal(knots, k2)
    cand = O.sample_sspp(ctrl0, 3, sigma, np.ones(7), seed, 0, B)
    arc, feas = O.sspp_score(osc, knots, 3, cand, W)
    fid = np.nonzero(feas)[0]
    assert list(ids) == list(fid)
    np.testing.assert_array_equal(ctrl, cand[fid])
    assert np.abs(arcs - arc[fid]).max(initial=0.0) <= 1e-12
    idx, bc = O.argmin(arc, feas)
    assert best[1] == idx and best[2] == len(fid)


def test_first_plan_prepass_runs_asynchronously(cuda):
    """The drop-in planner's first plan() creates its job with the hit-order pre-pass off the
    call's path: the call scans in gap / bisection order, the census lands on its own stream,
    and a later launch swaps the hit order in.  Every call equals the oracle, including a call
    that re-targets the job (new start / end) after the pre-pass landed but before it was
    applied — that call may take only the waypoint order, since the pre-pass's pair tables are
    the creation's reachable subset."""
    import time
    import sspp_amd as S
    from sspp_amd import _lib
    import ctypes as C
    L = _lib.lib()
    model = S.Model(ROBOCRANE)
    scene = S.Scene(model, 0, 7)
    osc = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7)
    s0 = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    e0 = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
    s1 = s0 + np.array([0, 0, 0.05, 0, 0, 0, 0])
    for retarget in (False, True):
        pl = C.c_void_p()
        _lib.check(L.sspp_planner_create(scene.handle, 7, C.byref(pl)), "planner create")
        try:
            B, W, n = 4096, 128, 10
            r = _planner_plan(L, pl, s0, e0, 0.08, B, W, n, 11)
            assert _prepass_state(L, pl) in (1, 2)  # running or landed, not applied yet
            _check_plan(osc, r, s0, e0, 0.08, B, W, n, 11)
            t0 = time.time()
            while _prepass_state(L, pl) != 2 and time.time() - t0 < 30:
                time.sleep(0.01)
            assert _prepass_state(L, pl) == 2
            st = s1 if retarget else s0
            r = _planner_plan(L, pl, st, e0, 0.08, B, W, n, 12)
            assert _prepass_state(L, pl) == 3  # applied at this call's launch
            _check_plan(osc, r, st, e0, 0.08, B, W, n, 12)
            v = C.c_int64()
            _lib.check(L.sspp_planner_get_option(pl, _lib.OPT_WP_ORDER, C.byref(v)), "wp order")
            assert v.value == 2
            _lib.check(L.sspp_planner_get_option(pl, _lib.OPT_ORDER, C.byref(v)), "pair order")
            assert v.value == (1 if retarget else 2)
            r = _planner_plan(L, pl, s0, e0, 0.1, B, W, n, 13)
            _check_plan(osc, r, s0, e0, 0.1, B, W, n, 13)
        finally:
            L.sspp_planner_free(pl)

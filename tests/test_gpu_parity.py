"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle on the same inputs.

Bars (BASELINE.json north_star): per-candidate costs within 1e-5 of the oracle — the kernels
follow the oracle's operation order, so the tests hold them to 1e-12 (SamplingPathPlanner)
and 1e-9 (TaskSpacePlanner: control points from the same Householder QR replay as the oracle;
costs summed in the canonical lane order); feasibility flags and the selected index
bit-identical.
"""
import os

import numpy as np
import pytest

from oracle import mjcf_ref
from oracle import oracle as O
from tests.conftest import SCENES, arc_err

pytestmark = pytest.mark.gpu

ROBOCRANE = os.path.join(SCENES, "robocrane.xml")
STACKING = os.path.join(SCENES, "stacking.xml")
PLANNER = os.path.join(SCENES, "planner.xml")
START7 = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
END7 = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
COST_TOL = 1e-12


def _np(t):
    return t.detach().cpu().numpy()


def linear_init(start, end, n, p=3):
    import sspp_amd as S
    u = np.array([i / (n - 1) for i in range(n)])
    pts = np.array([(1 - t) * start + t * end for t in u])
    return S.interpolate(pts, p, u)


@pytest.fixture(scope="module")
def robocrane(cuda):
    import sspp_amd as S
    model = S.Model(ROBOCRANE)
    scene = S.Scene(model, 0, 7)
    oscene = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7)
    return model, scene, oscene


def run_sspp(job, B, first=0, with_ctrl=True):
    import sspp_amd as S
    out = job.alloc(B, with_ctrl=with_ctrl)
    job.sample_score(first, B, out["arc"], out["feasible"], out["best"], ctrl_out=out.get("ctrl"))
    import torch
    torch.cuda.synchronize()
    res = {k: _np(v) for k, v in out.items() if k != "best"}
    res["best"] = S.decode_best(out["best"])
    return res


# k_sspp_c2f launch shapes (threads per workgroup, phase-1 lanes per candidate), forced through
# the job option SSPP_OPT_SHAPE_NT / _G1; (0, 0) = the shape the library picks per launch
# (256 x 64 below 16384 candidates per launch, 128 x 4 above).  Every shape must give the
# oracle's results.
SHAPES = [(0, 0), (128, 4), (64, 4), (64, 3), (64, 8), (64, 16), (64, 64), (256, 64), (256, 16)]


def set_shape(job, nt, g1):
    job.set_shape(nt, g1)


@pytest.mark.parametrize("arc_all", [False, True])
@pytest.mark.parametrize("nt,g1", SHAPES)
@pytest.mark.parametrize("B,W", [(4096, 128), (257, 128), (1, 128), (300, 50), (100, 256), (64, 2)])
def test_robocrane_sample_score_matches_oracle(robocrane, nt, g1, B, W, arc_all):
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), W, seed=0x5EED, max_batch=B,
                    arc_all=arc_all)
    set_shape(job, nt, g1)
    r = run_sspp(job, B, first=1000)
    # sampling parity (Philox + FP64 Box-Muller restated on the host): bit-identical
    ctrl_o = O.sample_sspp(ctrl0, 3, 0.08, np.ones(7), 0x5EED, 1000, B)
    assert np.array_equal(r["ctrl"], ctrl_o)
    # scoring parity on the exact control points the GPU scored
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], W, arc_all=arc_all)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert np.isinf(r["arc"]).sum() == (0 if arc_all else int((feas_o == 0).sum()))
    assert arc_err(r["arc"], arc_o) <= COST_TOL
    idx_o, best_o = O.argmin(arc_o, feas_o)
    cost, idx, cnt = r["best"]
    assert cnt == int(feas_o.sum())
    assert idx == (idx_o + 1000 if idx_o >= 0 else -1)
    if idx_o >= 0:
        assert abs(cost - best_o) <= COST_TOL


@pytest.mark.parametrize("nt,g1", [(128, 1), (256, 1), (256, 2), (256, 3)])
def test_oversized_shapes_are_refused(robocrane, nt, g1):
    """k_sspp_c2f reduces with one wave: a forced shape of more than 64 candidates per
    workgroup ((NT / 64) * (64 / G1) > 64) must fail loudly, not score a subset."""
    import sspp_amd as S
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=4096)
    set_shape(job, nt, g1)
    with pytest.raises(S.SsppError, match="more than 64 candidates"):
        run_sspp(job, 4096, with_ctrl=False)


def test_robocrane_config2_is_nontrivial(robocrane):
    """Config 2 must have both feasible and colliding candidates (else parity is vacuous)."""
    import sspp_amd as S
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=4096)
    r = run_sspp(job, 4096, with_ctrl=False)
    nfeas = int(r["feasible"].sum())
    assert 0 < nfeas < 4096, nfeas  # SURVEY config 2 (sigma 0.08): ~0.3% clear the brick stack


@pytest.mark.parametrize("nt,g1", SHAPES)
def test_score_ctrl_mode_matches_oracle(robocrane, nt, g1):
    """Caller-supplied splines (checkCollision + computeArcLength on arbitrary ctrl)."""
    import sspp_amd as S
    import torch
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    rng = np.random.default_rng(7)
    B = 777
    ctrl = ctrl0[None] + rng.normal(0, 0.05, size=(B, 10, 7))  # endpoints perturbed too
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=B)
    set_shape(job, nt, g1)
    out = job.alloc(B)
    job.score_ctrl(torch.from_numpy(ctrl).cuda(), 0, out["arc"], out["feasible"], out["best"])
    torch.cuda.synchronize()
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, ctrl, 128)
    np.testing.assert_array_equal(_np(out["feasible"]), feas_o)
    assert arc_err(_np(out["arc"]), arc_o) <= COST_TOL
    assert S.decode_best(out["best"])[1] == O.argmin(arc_o, feas_o)[0]


@pytest.mark.parametrize("nt,g1", [(0, 0), (128, 4), (64, 4), (256, 64)])
@pytest.mark.parametrize("sigma,B,W", [(0.08, 4096, 128), (0.2, 4096, 128), (0.08, 2048, 256)])
def test_fp32_filter_is_invisible(robocrane, nt, g1, sigma, B, W):
    """The FP32-filtered scan (SSPP_OPT_F32, default on; sspp_filter.h) against the all-FP64 scan
    on the same candidates: arcs, feasibility and the argmin record bit-identical, in sample mode
    and for caller splines (endpoints perturbed: positions and quaternions everywhere).  sigma 0.2
    puts many more candidates near contact than the bench's 0.08."""
    import sspp_amd as S
    import torch
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    res = {}
    for f32 in (1, 0):
        job = S.SsppJob(scene, knots, 3, ctrl0, sigma, np.ones(7), W, seed=0x5EED, max_batch=B)
        set_shape(job, nt, g1)
        job.set_option(S.OPT_F32, f32)
        r = run_sspp(job, B, first=3000)
        assert job.get_option(S._lib.OPT_LAST_F32) == f32  # the filter ran (or not)
        ctrl = ctrl0[None] + np.random.default_rng(11).normal(0, sigma, size=(B, 10, 7))
        out = job.alloc(B)
        job.score_ctrl(torch.from_numpy(ctrl).cuda(), 0, out["arc"], out["feasible"], out["best"])
        torch.cuda.synchronize()
        res[f32] = (r, _np(out["arc"]), _np(out["feasible"]), S.decode_best(out["best"]))
    (a, aarc, afeas, abest), (b, barc, bfeas, bbest) = res[1], res[0]
    np.testing.assert_array_equal(a["ctrl"], b["ctrl"])
    np.testing.assert_array_equal(a["feasible"], b["feasible"])
    np.testing.assert_array_equal(a["arc"], b["arc"])
    assert a["best"] == b["best"]
    np.testing.assert_array_equal(afeas, bfeas)
    np.testing.assert_array_equal(aarc, barc)
    assert abest == bbest
    assert 0 < int(a["feasible"].sum()) < B and 0 < int(afeas.sum()) < B  # both outcomes occur


def test_config1_bsplines_golden(cuda, golden):
    """Config 1: 2-DoF, 64 x 50, no collision, knots/ctrl from the reference's BSplines.py."""
    import sspp_amd as S
    import torch
    knots, ctrl = golden["cfg1_knots"], golden["cfg1_ctrl"]
    job = S.SsppJob(None, knots, 3, golden["cfg1_ctrl0"], 0.08, np.ones(2), 50, max_batch=64)
    out = job.alloc(64)
    job.score_ctrl(torch.from_numpy(np.ascontiguousarray(ctrl)).cuda(), 0, out["arc"],
                   out["feasible"], out["best"])
    torch.cuda.synchronize()
    arc = _np(out["arc"])
    assert np.abs(arc - golden["cfg1_arc"]).max() <= 1e-12
    arc_o, _ = O.sspp_score(None, knots, 3, ctrl, 50)
    assert np.abs(arc - arc_o).max() == 0.0
    assert S.decode_best(out["best"])[1] == int(golden["cfg1_best"][0])
    assert _np(out["feasible"]).all()


def test_robot_path_d9_p2_golden(cuda, golden):
    """The reference's robot path pipeline (scripts/main_bspline.py:198-209): a degree-2 spline
    through 7 via points in 9-D (knots [0,0,0,.2,.4,.6,.8,1,1,1]); control points from the
    reference's compute_control_points, arc length on 128 points from its bspline().  The GPU's
    computeArcLength of that spline equals the reference's to 1e-12 and the oracle's exactly."""
    import sspp_amd as S
    import torch
    knots, ctrl = golden["robot_knots"], golden["robot_ctrl"]
    job = S.SsppJob(None, knots, 2, ctrl, 0.0, np.ones(9), 128, max_batch=3)
    out = job.alloc(3)
    cands = np.stack([ctrl, ctrl * 0.5, ctrl[::-1]])
    job.score_ctrl(torch.from_numpy(np.ascontiguousarray(cands)).cuda(), 0, out["arc"], out["feasible"], out["best"])
    torch.cuda.synchronize()
    arc = _np(out["arc"])
    assert abs(arc[0] - golden["robot_arc"][0]) <= 1e-12
    arc_o, _ = O.sspp_score(None, knots, 2, cands, 128)
    assert np.array_equal(arc, arc_o)
    assert _np(out["feasible"]).all()


def test_reference_robot_path_fixture_on_gpu(cuda):
    """The reference's saved robot path (scripts/bspline_params.npy, main_bspline.py:198-209;
    fixture tests/golden/robot_path.json): D = 9, degree 2.  The GPU's computeArcLength equals
    the reference's BSplines.bspline chord sum to 1e-12 and the oracle's exactly, alone and
    among other candidates of the same launch (ragged batch of 5)."""
    import json
    import sspp_amd as S
    import torch
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "robot_path.json")))
    knots, ctrl = np.array(d["knots"]), np.array(d["ctrl"])
    job = S.SsppJob(None, knots, 2, ctrl, 0.0, np.ones(9), d["W"], max_batch=5)
    cands = np.stack([ctrl, ctrl[::-1], ctrl * 0.5, ctrl + 0.1, ctrl])
    out = job.alloc(5)
    job.score_ctrl(torch.from_numpy(np.ascontiguousarray(cands)).cuda(), 0, out["arc"], out["feasible"],
                   out["best"])
    torch.cuda.synchronize()
    arc = _np(out["arc"])
    assert abs(arc[0] - d["arc_length"]) <= 1e-12 and arc[4] == arc[0]
    arc_o, _ = O.sspp_score(None, knots, 2, cands, d["W"])
    assert np.array_equal(arc, arc_o)
    assert S.decode_best(out["best"])[1] == O.argmin(arc_o, np.ones(5, np.uint8))[0]


def test_non_finite_arc_is_never_best(cuda):
    """findBestPath (include/sspp.h:171-192) takes a path only when its cost is below the running
    minimum from +inf: feasible candidates with an infinite or NaN arc length count as feasible
    but are never selected — on the device argmin as in the oracle."""
    import sspp_amd as S
    import torch
    knots, ctrl0 = linear_init(np.zeros(2), np.ones(2), 10)
    B = 300
    rng = np.random.default_rng(5)
    ctrl = ctrl0[None] + rng.normal(0, 0.05, size=(B, 10, 2))
    ctrl[0, 4, 0] = np.inf     # lowest ids: would win a tie-break if they were eligible
    ctrl[1, 5, 1] = np.nan
    ctrl[2:7] *= 1e300         # arc overflows to +inf
    job = S.SsppJob(None, knots, 3, ctrl0, 0.0, np.ones(2), 50, max_batch=B)
    out = job.alloc(B)
    job.score_ctrl(torch.from_numpy(ctrl).cuda(), 0, out["arc"], out["feasible"], out["best"])
    torch.cuda.synchronize()
    arc = _np(out["arc"])
    assert not np.isfinite(arc[:7]).any() and np.isfinite(arc[7:]).all()
    idx_o, best_o = O.argmin(arc, np.ones(B, np.uint8))
    cost, idx, cnt = S.decode_best(out["best"])
    assert idx == idx_o >= 7 and cost == best_o and cnt == B


def stacking_problem(B, cp=128, seed=0x5EED, K=1):
    import sspp_amd as S
    model = S.Model(STACKING)
    scene = S.Scene(model, 1, "block1")
    start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
    end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
    mean = np.array([start + (end - start) * (i + 1) / (K + 1) for i in range(K)])
    sigma = np.full((K, 4), 0.2)
    lo, hi = np.array([-0.5, -0.5, 0.0, -1.6]), np.array([0.5, 0.5, 0.6, 1.6])
    job = S.TspJob(scene, start, end, K, cp, mean=mean, sigma=sigma, lo=lo, hi=hi, z_min=0.0,
                   seed=seed, max_batch=B)
    oscene = O.Scene(mjcf_ref.load(STACKING), 1, model.body_id("block1"))
    return model, scene, job, oscene, start, end, mean, sigma, lo, hi


@pytest.mark.parametrize("form", [-1, 0])
@pytest.mark.parametrize("B,cp,K", [(16384, 128, 1), (333, 40, 1), (200, 64, 3), (50, 300, 2), (1000, 256, 1)])
def test_stacking_tsp_matches_oracle(cuda, B, cp, K, form):
    """form -1: the library's choice (k_tsp with deferred box-box polygons where it applies:
    one waypoint per lane), 0: the inline k_tsp."""
    import sspp_amd as S
    import torch
    model, scene, job, oscene, start, end, mean, sigma, lo, hi = stacking_problem(B, cp, K=K)
    job.set_option(S.OPT_TSP_FORM, form)
    out = job.alloc(B, with_vias=True)
    job.sample_score(5, B, out["L"], out["Cnf"], out["Cwf"], out["status"], out["cost"],
                     out["best"], vias_out=out["vias"])
    torch.cuda.synchronize()
    vias = _np(out["vias"])
    vias_o = O.sample_tsp(mean, sigma, lo, hi, 0.0, 0x5EED, 5, B)
    assert np.abs(vias - vias_o).max() <= 1e-12
    L, Cnf, Cwf, st, cost = O.tsp_score(oscene, start, end, vias, cp)
    np.testing.assert_array_equal(_np(out["status"]), st)
    for a, b in ((out["L"], L), (out["Cnf"], Cnf), (out["Cwf"], Cwf), (out["cost"], cost)):
        assert np.abs(_np(a) - b).max() <= 1e-9
    idx_o, best_o = O.tsp_best(cost, st)
    c, idx, cnt = S.decode_best(out["best"])
    assert cnt == int(st.sum())
    assert idx == (idx_o + 5 if idx_o >= 0 else -1)
    if B >= 1000:
        assert 0 < st.sum() < B  # both outcomes present
    if form < 0 and cp <= 256 and B > 512:
        assert job.get_option(S.OPT_TSP_FORM) == 3  # the deferred form ran


@pytest.mark.parametrize("nt,g1", SHAPES)
def test_planner_scene_sspp(cuda, nt, g1):
    """planner.xml: block1 (free) vs static wall/block2, 7-DoF window, path through the wall."""
    import sspp_amd as S
    model = S.Model(PLANNER)
    scene = S.Scene(model, 0, 7)
    oscene = O.Scene(mjcf_ref.load(PLANNER), 0, 7)
    start = np.array([0.5, 0.0, 0.15, 1, 0, 0, 0])
    end = np.array([-0.25, 0.0, 0.15, 1, 0, 0, 0])
    knots, ctrl0 = linear_init(start, end, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.3, np.array([1, 1, 1, .2, .2, .2, .2]), 100,
                    seed=3, max_batch=2048)
    set_shape(job, nt, g1)
    r = run_sspp(job, 2048)
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], 100)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert arc_err(r["arc"], arc_o) <= COST_TOL
    assert r["best"][1] == O.argmin(arc_o, feas_o)[0]


@pytest.mark.parametrize("nt,g1", SHAPES)
def test_cylinder_box_sspp(robocrane, nt, g1):
    """The block grazing the gripper's col_mount cylinder cap (and col_base box): the scan loops
    leave cylinder-box pairs that pass the bounding-sphere test undecided, and k_sspp_c2f's
    settle step (the exact test, out of line, same launch) decides them for the candidates with
    no other contact.  Feasibility, arcs and the argmin must equal the oracle's exact test."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(GRAZE_START, GRAZE_END, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.01, GRAZE_LIMITS, 128, seed=11, max_batch=2048)
    assert job.config()["cylinder_box"]
    set_shape(job, nt, g1)
    r = run_sspp(job, 2048)
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], 128)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert 0 < feas_o.sum() < 2048
    assert arc_err(r["arc"], arc_o) <= COST_TOL
    assert r["best"][1] == O.argmin(arc_o, feas_o)[0]
    # the cylinder-box pair decides some candidates: without it they would be feasible
    oscene_nocyl = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7, skip_types=(5,))
    _, feas_nc = O.sspp_score(oscene_nocyl, knots, 3, r["ctrl"], 128)
    assert (feas_nc.astype(int) - feas_o.astype(int)).max() == 1


GRAZE_START = np.array([1.8, 2.2, 0.656, 1, 0, 0, 0])
GRAZE_END = np.array([2.2, 2.2, 0.656, 1, 0, 0, 0])
GRAZE_LIMITS = np.array([1, 1, 1, .2, .2, .2, .2])


@pytest.mark.parametrize("spl", [3, 16])
def test_cylinder_box_multistep(robocrane, spl):
    """The grazing cylinder-box workload through the step executor (SsppSteps, G = 19 steps,
    spl steps per launch, 2 streams): step > 0 indexing of the settle step's exact decisions.
    Every step's argmin record and its per-candidate feasibility equal the oracle on that
    step's candidates, and some candidates turn on the cylinder-box pair."""
    import sspp_amd as S
    import torch
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(GRAZE_START, GRAZE_END, 10)
    B, G, stride, first = 1024, 19, 3 * 1024, 7 * 1024
    jobs = [S.SsppJob(scene, knots, 3, ctrl0, 0.01, GRAZE_LIMITS, 128, seed=11, max_batch=B) for _ in range(2)]
    arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda") for _ in jobs]
    feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda") for _ in jobs]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    ex = S.SsppSteps(jobs, streams, B, arcs, feas, steps_per_launch=spl)
    best = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    ex.enqueue(G, first, stride, best)
    torch.cuda.synchronize()
    got = best.cpu()
    oscene_nocyl = O.Scene(mjcf_ref.load(ROBOCRANE), 0, 7, skip_types=(5,))
    turned = 0
    for i in range(G):
        ctrl = O.sample_sspp(ctrl0, 3, 0.01, GRAZE_LIMITS, 11, first + i * stride, B)
        arc_o, feas_o = O.sspp_score(oscene, knots, 3, ctrl, 128)
        idx_o, best_o = O.argmin(arc_o, feas_o)
        cost, idx, cnt = S.decode_best(got[i])
        assert cnt == int(feas_o.sum()), i
        assert idx == (idx_o + first + i * stride if idx_o >= 0 else -1), i
        if idx_o >= 0:
            assert abs(cost - best_o) <= COST_TOL
        _, feas_nc = O.sspp_score(oscene_nocyl, knots, 3, ctrl, 128)
        turned += int((feas_nc.astype(int) - feas_o.astype(int)).max() == 1)
        if i % (2 * spl) < spl and i // spl == (G - 1) // spl:  # the last launch of branch 0
            pass
    assert turned > 0
    # per-candidate feasibility of the last launch on branch 0 (its scratch outputs)
    last0 = max(l for l in range((G + spl - 1) // spl) if l % 2 == 0)
    for k in range(min(spl, G - last0 * spl)):
        i = last0 * spl + k
        ctrl = O.sample_sspp(ctrl0, 3, 0.01, GRAZE_LIMITS, 11, first + i * stride, B)
        _, feas_o = O.sspp_score(oscene, knots, 3, ctrl, 128)
        np.testing.assert_array_equal(feas[0][k * B:(k + 1) * B].cpu().numpy(), feas_o)


@pytest.mark.parametrize("nt,g1", [(0, 0), (64, 4)])
def test_fused_argmin_back_to_back(robocrane, nt, g1):
    """100 batches queued back to back: each launch's in-kernel argmin (sharded arrival
    counters, re-armed by the last workgroup) must equal the argmin of that batch's outputs."""
    import sspp_amd as S
    import torch
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    B, steps = 4096, 100
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.12, np.ones(7), 128, max_batch=B)
    set_shape(job, nt, g1)
    arc = torch.empty((steps, B), dtype=torch.float64, device="cuda")
    feas = torch.empty((steps, B), dtype=torch.uint8, device="cuda")
    best = torch.empty((steps, 4), dtype=torch.int64, device="cuda")
    for i in range(steps):
        job.sample_score(i * B, B, arc[i], feas[i], best[i])
    torch.cuda.synchronize()
    arc, feas = _np(arc), _np(feas)
    for i in range(steps):
        idx, c = O.argmin(arc[i], feas[i])
        cost, bi, cnt = S.decode_best(best[i])
        assert cnt == int(feas[i].sum())
        assert bi == (idx + i * B if idx >= 0 else -1)
        if idx >= 0:
            assert cost == c
    # same candidates as the separate sampler: compare one batch against the oracle sampler
    r = run_sspp(job, 257, first=77)
    assert np.abs(r["ctrl"] - O.sample_sspp(ctrl0, 3, 0.12, np.ones(7), 0x5EED, 77, 257)).max() <= 1e-12


@pytest.mark.parametrize("spl", [1, 3, 16, 20, 32])
def test_step_executor_matches_eager(robocrane, spl):
    """C++ step executor: G steps, spl per launch, launches round robin over 3 streams; every
    step's argmin record equals a single eager launch on the same candidate ids."""
    import sspp_amd as S
    import torch
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    B, G, stride, first = 4096, 19, 2 * 4096, 5 * 4096
    jobs = [S.SsppJob(scene, knots, 3, ctrl0, 0.12, np.ones(7), 128, max_batch=B) for _ in range(3)]
    arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda") for _ in jobs]
    feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda") for _ in jobs]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(2)]
    ex = S.SsppSteps(jobs, streams, B, arcs, feas, steps_per_launch=spl)
    best = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    ex.enqueue(G, first, stride, best)
    torch.cuda.synchronize()
    got = best.cpu()
    ref = jobs[0].alloc(B)
    for i in range(G):
        jobs[0].sample_score(first + i * stride, B, ref["arc"], ref["feasible"], ref["best"])
        torch.cuda.synchronize()
        assert S.decode_best(got[i]) == S.decode_best(ref["best"]), i


# split: whether the launch must run the split instance (survivor queue): single-geom sampled
# tables (sigma <= 0.12) whose grid is one resident round of MI355X's 256 CUs (10 two-wave
# workgroups each: 20 steps x 128 workgroups fit, 32 steps do not)
@pytest.mark.parametrize("sigma,spl,split", [(0.08, 20, 1), (0.08, 32, 0), (0.02, 16, 1), (0.3, 20, 0)])
def test_multistep_launch_matches_oracle(robocrane, sigma, spl, split):
    """The executor's launches of many steps (the one-wave throughput shape, the bench's launch):
    every step's per-candidate feasibility and arc length equal the oracle's on the same Philox
    candidates, and every step's argmin record the oracle's argmin, over two launches back to
    back (re-armed argmin counters).  sigma 0.02 leaves most candidates surviving phase 1,
    sigma 0.3 almost none."""
    import sspp_amd as S
    import torch
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    B, G, stride, first = 4096, spl, 4096, 7 * 4096
    job = S.SsppJob(scene, knots, 3, ctrl0, sigma, np.ones(7), 128, max_batch=B)
    arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda")]
    feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda")]
    ex = S.SsppSteps([job], [torch.cuda.current_stream()], B, arcs, feas, steps_per_launch=spl)
    best = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    for rep in range(2):
        ex.enqueue(G, first + rep * G * stride, stride, best)
        torch.cuda.synchronize()
        assert job.config()["shape"] == "128x4"
        assert job.get_option(S._lib.OPT_LAST_SPLIT) == split
        arc, fe, got = arcs[0].cpu().numpy(), feas[0].cpu().numpy(), best.cpu()
        for i in (0, 7, G - 1):
            f0 = first + (rep * G + i) * stride
            ctrl = O.sample_sspp(ctrl0, 3, sigma, np.ones(7), 0x5EED, f0, B)
            arc_o, feas_o = O.sspp_score(oscene, knots, 3, ctrl, 128)
            np.testing.assert_array_equal(fe[i * B:(i + 1) * B], feas_o)
            assert arc_err(arc[i * B:(i + 1) * B], arc_o) <= COST_TOL
            k, _ = O.argmin(arc_o, feas_o)
            d = S.decode_best(got[i])
            assert d[1] == (f0 + k if k >= 0 else -1) and d[2] == int(feas_o.sum()), (rep, i, d, k)


def test_default_shape_single_step_matches_oracle(robocrane):
    """BASELINE configs[1] exactly as a plan() batch runs it: 4096 x 128, no forced shape (the
    library picks the latency shape, 256 x 64), hit order from the creation pre-pass; every
    candidate against the oracle."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=4096)
    r = run_sspp(job, 4096, first=12345)
    cfg = job.config()
    assert cfg["shape"] == "256x64" and cfg["pair_order"] == "hit" and cfg["waypoint_order"] == "hit"
    assert np.array_equal(r["ctrl"], O.sample_sspp(ctrl0, 3, 0.08, np.ones(7), 0x5EED, 12345, 4096))
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], 128)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert arc_err(r["arc"], arc_o) <= COST_TOL
    k, _ = O.argmin(arc_o, feas_o)
    assert r["best"][1] == (12345 + k if k >= 0 else -1) and r["best"][2] == int(feas_o.sum())


def test_environment_does_not_change_results(robocrane, monkeypatch):
    """The library reads no environment variables: names that earlier builds read (sampler,
    ablation, kernel and shape switches) leave a default job's results unchanged."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)

    def run():
        job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=2048)
        return run_sspp(job, 2048, first=777), job.config()

    base, cfg0 = run()
    for k, v in dict(SSPP_SAMPLER="1", SSPP_ABLATE="64", SSPP_KERNEL="2", SSPP_G1="16", SSPP_NT="128",
                     SSPP_PAIR_ORDER="0", SSPP_REACH="0", SSPP_HULL="0", SSPP_INSAMPLE="0").items():
        monkeypatch.setenv(k, v)
    again, cfg1 = run()
    cfg0.pop("prepass_ms"), cfg1.pop("prepass_ms")  # host timing
    assert cfg0 == cfg1 and cfg0["sampler"] == "fp64"
    for k in ("ctrl", "arc", "feasible"):
        assert np.array_equal(base[k], again[k]), k
    assert base["best"] == again["best"]
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, base["ctrl"], 128)
    np.testing.assert_array_equal(base["feasible"], feas_o)


@pytest.mark.parametrize("nt,g1", [(0, 0), (64, 4)])
def test_fp32_sampler_opt_in(robocrane, nt, g1):
    """The opt-in FP32 Box-Muller quads (sampler = 1): candidates bit-identical to the oracle's
    or_normal_quad, scoring parity as with the FP64 default, and the two samplers differ."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    B = 1500
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=B, sampler=S.SAMPLER_FP32)
    set_shape(job, nt, g1)
    assert job.config()["sampler"] == "fp32"
    r = run_sspp(job, B, first=321)
    want = O.sample_sspp(ctrl0, 3, 0.08, np.ones(7), 0x5EED, 321, B, sampler=O.SAMPLER_FP32)
    assert np.array_equal(r["ctrl"], want)
    assert not np.array_equal(want, O.sample_sspp(ctrl0, 3, 0.08, np.ones(7), 0x5EED, 321, B))
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], 128)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert arc_err(r["arc"], arc_o) <= COST_TOL


def test_reduce_best_steps(cuda):
    import sspp_amd as S
    import torch
    rng = np.random.default_rng(3)
    R, G = 3, 9
    recs = np.zeros((R, G, 4), np.int64)
    for r in range(R):
        for g in range(G):
            c = rng.choice([0.5, 0.25, np.inf])
            idx = -1 if np.isinf(c) else int(rng.integers(0, 100))
            recs[r, g, 0] = np.array([c]).view(np.int64)[0]
            recs[r, g, 1] = idx
            recs[r, g, 2] = int(rng.integers(0, 5))
    out = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    S.reduce_best_steps(torch.from_numpy(recs).cuda(), out)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    for g in range(G):
        cands = [(recs[r, g, :1].view(np.float64)[0], recs[r, g, 1]) for r in range(R) if recs[r, g, 1] >= 0]
        want = min(cands) if cands else (np.inf, -1)
        cost, idx, cnt = S.decode_best(out[g])
        assert (cost, idx) == (float(want[0]), int(want[1]))
        assert cnt == int(recs[:, g, 2].sum())


def test_config4_full_size_shards(robocrane):
    """BASELINE configs[3] at full size on one GPU: 262144 candidates x 256 waypoints scored
    as one batch and as the 8 per-GPU shards of 32768 (global Philox ids) give identical
    per-candidate results, and the 8 shard records reduce to the whole batch's argmin (the
    RCCL all-gather path).  A random 512-candidate subset is checked against the oracle."""
    import sspp_amd as S
    import torch
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    B, W, R = 262144, 256, 8
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), W, max_batch=B)
    whole = job.alloc(B, with_ctrl=True)
    job.sample_score(0, B, whole["arc"], whole["feasible"], whole["best"], ctrl_out=whole["ctrl"])
    per = B // R
    arc = torch.empty(B, dtype=torch.float64, device="cuda")
    feas = torch.empty(B, dtype=torch.uint8, device="cuda")
    recs = torch.zeros((R, 4), dtype=torch.int64, device="cuda")
    for r in range(R):
        job.sample_score(r * per, per, arc[r * per:(r + 1) * per], feas[r * per:(r + 1) * per], recs[r])
    out = S.best_tensor()
    S.reduce_best_device(recs, out)
    torch.cuda.synchronize()
    assert torch.equal(arc, whole["arc"]) and torch.equal(feas, whole["feasible"])
    assert S.decode_best(out) == S.decode_best(whole["best"])
    cost, idx, cnt = S.decode_best(whole["best"])
    a, f = _np(whole["arc"]), _np(whole["feasible"])
    assert cnt == int(f.sum()) and 0 < cnt < B
    assert idx == O.argmin(a, f)[0] and cost == a[idx]
    sub = np.sort(np.random.default_rng(0).choice(B, 512, replace=False))
    sub = np.union1d(sub, [idx])
    ctrl = _np(whole["ctrl"][torch.from_numpy(sub).cuda()])
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, ctrl, W)
    np.testing.assert_array_equal(f[sub], feas_o)
    assert arc_err(a[sub], arc_o) <= COST_TOL


@pytest.mark.parametrize("order", [0, 1, 2])
def test_scan_orders_identical(robocrane, order):
    """The pair / waypoint scan order (SSPP_OPT_ORDER: scene + bisection, mean-path gap, hit
    order) steers only how soon a contact is found: per-candidate results equal the oracle."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=2048)
    job.set_option(S.OPT_ORDER, order)
    r = run_sspp(job, 2048, first=4096)
    arc_o, feas_o = O.sspp_score(oscene, knots, 3, r["ctrl"], 128)
    np.testing.assert_array_equal(r["feasible"], feas_o)
    assert arc_err(r["arc"], arc_o) <= COST_TOL
    assert r["best"][1] == (O.argmin(arc_o, feas_o)[0] + 4096 if feas_o.any() else -1)


@pytest.mark.parametrize("goal", [0, 3, 5])
def test_gripper_tsp_matches_oracle(cuda, goal):
    """Multi-geom mover (robocrane gripper: 7 collidable geoms, k_tsp<1, false>, lazy geom
    rotation, exact plane cull): per-candidate L / C_nf / C_wf / cost and status vs the oracle
    on the device's own via sets; the multi-goal bench scenarios (BASELINE configs[4])."""
    import sspp_amd as S
    import torch
    import bench
    model = S.Model(ROBOCRANE)
    body = model.body_id("gripper_collision_with_block/")
    scene = S.Scene(model, 1, body)
    oscene = O.Scene(mjcf_ref.load(ROBOCRANE), 1, body)
    start, end = (np.array(x) for x in bench.MULTIGOAL[goal])
    B, cp = 3000, 96
    mean = (start + 0.5 * (end - start)).reshape(1, 4)
    sigma = np.array([[0.15, 0.15, 0.15, 0.5]])
    job = S.TspJob(scene, start, end, 1, cp, mean=mean, sigma=sigma, lo=bench.MG_LO,
                   hi=bench.MG_HI, max_batch=B)
    out = job.alloc(B, with_vias=True)
    job.sample_score(0, B, out["L"], out["Cnf"], out["Cwf"], out["status"], out["cost"],
                     out["best"], vias_out=out["vias"])
    torch.cuda.synchronize()
    vias = _np(out["vias"])
    L, Cnf, Cwf, st, cost = O.tsp_score(oscene, start, end, vias, cp)
    np.testing.assert_array_equal(_np(out["status"]), st)
    for a, b in ((out["L"], L), (out["Cnf"], Cnf), (out["Cwf"], Cwf), (out["cost"], cost)):
        assert np.abs(_np(a) - b).max() <= 1e-9
    assert 0 < st.sum() < B  # both outcomes present
    assert S.decode_best(out["best"])[1] == O.tsp_best(cost, st)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("xml,body,B,cp", [("robocrane.xml", "gripper_collision_with_block/", 17, 40),
                                           ("robocrane.xml", "gripper_collision_with_block/", 300, 64),
                                           ("stacking.xml", "block1", 200, 48)])
def test_tsp_kernel_forms_identical(cuda, xml, body, B, cp):
    """k_tsp, the single-workgroup pair split (k_tsp_pp), the multi-workgroup split (k_tsp_pp2,
    48 gripper pairs over 6 workgroups per candidate) and the two deferred-polygon forms of k_tsp
    (3: compacted per workgroup, <= 8 pairs; 4: summed per lane after its pair loop, the gripper's
    48 pairs) give bit-identical per-candidate results and argmin records, and match the oracle.
    A form that does not apply to a scene runs k_tsp (the read-back says which ran)."""
    import torch
    import sspp_amd as S
    path = os.path.join(SCENES, xml)
    model = S.Model(path)
    bid = model.body_id(body)
    scene = S.Scene(model, 1, bid)
    if xml == "robocrane.xml":
        start, end = np.array([0.5, 0.15, 0.156, 1.5708]), np.array([0.5, -0.05, 0.156, 1.5708])
        lo, hi = (0.0, -0.7, 0.1, -1.6), (0.7, 0.7, 0.6, 1.6)
    else:
        start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
        end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
        lo, hi = (-0.5, -0.5, 0.0, -1.6), (0.5, 0.5, 0.6, 1.6)
    mean = (start + 0.5 * (end - start)).reshape(1, 4)
    sigma = np.full((1, 4), 0.15)
    job = S.TspJob(scene, start, end, 1, cp, mean=mean, sigma=sigma, lo=np.array(lo), hi=np.array(hi),
                   z_min=0.0, max_batch=B)
    res = {}
    for mode in ("0", "1", "2", "3", "4"):
        job.set_option(S.OPT_TSP_FORM, int(mode))
        q = job.alloc(B, device="cuda", with_vias=True)
        job.sample_score(0, B, q["L"], q["Cnf"], q["Cwf"], q["status"], q["cost"], q["best"],
                         vias_out=q["vias"])
        torch.cuda.synchronize()
        res[mode] = {k: v.cpu().numpy() for k, v in q.items()}
    for mode in ("1", "2", "3", "4"):
        for k in ("L", "Cnf", "Cwf", "cost", "status", "vias", "best"):
            np.testing.assert_array_equal(res[mode][k], res["0"][k], err_msg="%s %s" % (mode, k))
    osc = O.Scene(mjcf_ref.load(path), 1, bid)
    L, Cnf, Cwf, st, cost = O.tsp_score(osc, start, end, res["0"]["vias"], cp)
    np.testing.assert_array_equal(res["0"]["status"], st)
    fin = np.isfinite(cost)
    assert (np.abs(res["0"]["cost"][fin] - cost[fin]) <= 1e-12 * np.maximum(1.0, np.abs(cost[fin]))).all()


@pytest.mark.parametrize("sigma,spl,B", [(0.08, 20, 4096), (0.02, 16, 4096), (0.12, 4, 8192), (0.3, 40, 1024)])
def test_split_launch_is_invisible(robocrane, sigma, spl, B):
    """Split launches (SSPP_OPT_SPLIT, default: every workgroup of k_sspp_c2f queues its phase-1
    survivors and every wave finishes queued survivors) against unsplit launches of the same
    steps: every output bit-identical — arcs, feasibility and each step's argmin record — over
    three launches back to back on two streams (the queue re-armed by each launch's last
    workgroup).  sigma 0.02 leaves most candidates surviving phase 1, 0.3 almost none; at 0.3
    the sampled pair table reaches more than one geom, which run_sspp never splits."""
    import sspp_amd as S
    import torch
    _, scene, _ = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    G, stride, first = 3 * spl, B, 11 * B
    out = {}
    for split in (1, 0):
        jobs = [S.SsppJob(scene, knots, 3, ctrl0, sigma, np.ones(7), 128, max_batch=B) for _ in range(2)]
        for j in jobs:
            j.set_option(S.OPT_SPLIT, split)
        arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda") for _ in jobs]
        feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda") for _ in jobs]
        streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
        ex = S.SsppSteps(jobs, streams, B, arcs, feas, steps_per_launch=spl)
        best = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
        ex.enqueue(G, first, stride, best)
        torch.cuda.synchronize()
        assert jobs[0].get_option(S._lib.OPT_LAST_SPLIT) == (split if sigma <= 0.12 else 0)
        # the last launch of each branch left its outputs in that branch's buffers
        out[split] = (best.cpu().numpy(), [a.cpu().numpy() for a in arcs], [f.cpu().numpy() for f in feas])
    (b1, a1, f1), (b0, a0, f0) = out[1], out[0]
    np.testing.assert_array_equal(b1, b0)
    for x, y in zip(a1, a0):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(f1, f0):
        np.testing.assert_array_equal(x, y)
    if sigma >= 0.08:  # (sigma 0.02 stays near the infeasible straight path: nothing feasible)
        assert (b1[:, 2] > 0).any()


@pytest.mark.parametrize("rep", [2, 3, 8])
def test_tsp_rep_is_invisible(cuda, rep):
    """SSPP_OPT_TSP_REP (k_tsp sub-batches per workgroup, one prologue for all of them) against
    one sub-batch per workgroup: every output bit-identical, the argmin record included, on a
    ragged batch (not a multiple of the workgroup's candidates)."""
    import sspp_amd as S
    import torch
    model = S.Model(os.path.join(SCENES, "stacking.xml"))
    scene = S.Scene(model, 1, "block1")
    start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
    end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
    mean = (start + 0.5 * (end - start)).reshape(1, 4)
    sigma = np.full((1, 4), 0.2)
    lo, hi = np.array([-0.5, -0.5, 0.0, -1.6]), np.array([0.5, 0.5, 0.6, 1.6])
    B = 3001
    res = {}
    for r in (1, rep):
        job = S.TspJob(scene, start, end, 1, 128, mean=mean, sigma=sigma, lo=lo, hi=hi, z_min=0.0, max_batch=B)
        job.set_option(S.OPT_TSP_REP, r)
        q = job.alloc(B)
        job.sample_score(77, B, q["L"], q["Cnf"], q["Cwf"], q["status"], q["cost"], q["best"])
        torch.cuda.synchronize()
        assert job.get_option(S.OPT_TSP_REP) == r
        res[r] = {k: v.cpu().numpy() for k, v in q.items()}
    for k in res[1]:
        np.testing.assert_array_equal(res[rep][k], res[1][k], err_msg=k)


def _split_run(job, spl, first, B=4096):
    """One split launch of spl steps through the executor: (arc, feas, records) on the host."""
    import sspp_amd as S
    import torch
    arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda")]
    feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda")]
    ex = S.SsppSteps([job], [torch.cuda.current_stream()], B, arcs, feas, steps_per_launch=spl)
    best = torch.zeros((spl, 4), dtype=torch.int64, device="cuda")
    ex.enqueue(spl, first, B, best)
    torch.cuda.synchronize()
    assert job.get_option(S._lib.OPT_LAST_SPLIT) == 1
    return arcs[0].cpu().numpy(), feas[0].cpu().numpy(), best.cpu().numpy()


def _split_vs_oracle(oscene, knots, ctrl0, sigma, spl, first, arc, fe, recs, steps, B=4096):
    import sspp_amd as S
    for i in steps:
        f0 = first + i * B
        ctrl = O.sample_sspp(ctrl0, 3, sigma, np.ones(7), 0x5EED, f0, B)
        arc_o, feas_o = O.sspp_score(oscene, knots, 3, ctrl, 128)
        np.testing.assert_array_equal(fe[i * B:(i + 1) * B], feas_o)
        assert arc_err(arc[i * B:(i + 1) * B], arc_o) <= COST_TOL
        k, _ = O.argmin(arc_o, feas_o)
        d = S.decode_best(recs[i])
        assert d[1] == (f0 + k if k >= 0 else -1) and d[2] == int(feas_o.sum()), (i, d, k)


def test_split_handoff_is_invisible(robocrane):
    """SSPP_OPT_SPLIT_LINGER_US = 0: every ticket that would wait for a slot not reserved yet is
    handed to the launch's last workgroup at once (the path a waiter takes after its linger
    expires).  Nothing is lost: the handed-over survivors are finished there, every output equals
    the default-linger launch bit for bit and the oracle, and no record reports lost work."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    spl, first = 20, 31 * 4096
    res = {}
    for linger in (0, 10000):
        job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=4096)
        job.set_option(S._lib.OPT_SPLIT_LINGER_US, linger)
        for rep in range(2):  # the second launch reuses the re-armed queue
            res[linger, rep] = _split_run(job, spl, first + rep * spl * 4096)
        res[linger, "handoffs"] = job.get_option(S._lib.OPT_SPLIT_HANDOFFS)
        assert job.get_option(S._lib.OPT_SPLIT_LOST) == 0
    assert res[0, "handoffs"] > 0  # the hand-over path ran
    for rep in range(2):
        for a, b in zip(res[0, rep], res[10000, rep]):
            np.testing.assert_array_equal(a, b)
        S.check_records(res[0, rep][2])
    arc, fe, recs = res[0, 1]
    _split_vs_oracle(oscene, knots, ctrl0, 0.08, spl, first + spl * 4096, arc, fe, recs, (0, 9, spl - 1))


def test_split_lost_work_fails_loudly_and_does_not_poison(robocrane):
    """SSPP_OPT_SPLIT_DROP (tests only) makes the last workgroup drop the handed-over survivors:
    the launch's lost-work check must report them in every step record (`reserved`), the Python
    layer must refuse those records (SsppError, SSPP_E_INCOMPLETE) and the job must count them.
    The next normal launch on the same queue must equal the oracle bit for bit: the last
    workgroup re-arms every reserved slot, so nothing stale reaches the next launch."""
    import sspp_amd as S
    _, scene, oscene = robocrane
    knots, ctrl0 = linear_init(START7, END7, 10)
    spl, first = 20, 53 * 4096
    job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=4096)
    job.set_option(S._lib.OPT_SPLIT_LINGER_US, 0)
    job.set_option(S._lib.OPT_SPLIT_DROP, 1)
    _, _, recs = _split_run(job, spl, first)
    lost = job.get_option(S._lib.OPT_SPLIT_LOST)
    assert lost > 0 and (recs[:, 3] == lost).all()
    with pytest.raises(S.SsppError, match="lost candidates"):
        S.decode_best(recs[0])
    with pytest.raises(S.SsppError, match="lost candidates"):
        S.check_records(recs)
    job.set_option(S._lib.OPT_SPLIT_DROP, 0)
    job.set_option(S._lib.OPT_SPLIT_LINGER_US, 10000)
    first2 = first + spl * 4096
    arc, fe, recs = _split_run(job, spl, first2)
    assert (recs[:, 3] == 0).all() and job.get_option(S._lib.OPT_SPLIT_LOST) == lost
    _split_vs_oracle(oscene, knots, ctrl0, 0.08, spl, first2, arc, fe, recs, range(spl))

"""Generate golden vectors from the reference's own Python operator API.

Run ONLY in the build container (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

It imports /root/reference/sspp/BSplines.py (with `casadi` stubbed: its NumPy functions
never touch CasADi — SURVEY §8c) and /root/reference/sspp/CubicPath.py, evaluates them,
and writes tests/golden/bsplines_golden.npz (inputs + outputs only, no reference source).

Fixture contents (SURVEY §8c list):
  knot_vector(n, k) for several (n, k)
  B / dB tables on a theta grid including 0, 1-1e-9 and 1
  compute_control_points for seeded random via points (n = 7, 10; d = 2, 7, 9)
  config 1: 64 candidates x 10 ctrl x 2-D, 50 waypoints via bspline(), arc lengths, argmin
  CubicPath positions / velocities / accelerations on u in [-0.1, 1.1]
"""
import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference/sspp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bsplines_golden.npz")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    sys.modules.setdefault("casadi", types.ModuleType("casadi"))
    bs = _load("ref_BSplines", os.path.join(REF, "BSplines.py"))
    cpm = _load("ref_CubicPath", os.path.join(REF, "CubicPath.py"))
    out = {}

    # (i) knot vectors
    nk = [(3, 2), (5, 2), (5, 3), (7, 1), (7, 3), (10, 3), (10, 2)]
    out["kv_nk"] = np.array(nk, np.int64)
    for n, k in nk:
        out["kv_%d_%d" % (n, k)] = np.asarray(bs.knot_vector(n, k), np.float64)

    # (ii) basis tables
    thetas = np.concatenate([np.linspace(0, 1, 41), [1 - 1e-9, 0.999999, 1e-9, 0.5 + 1e-12]])
    out["basis_theta"] = thetas
    for n, k in [(5, 3), (10, 3), (7, 2), (7, 1)]:
        t = bs.knot_vector(n, k)
        out["B_%d_%d" % (n, k)] = np.array([[bs.B(th, k, i, t) for i in range(n)] for th in thetas])
        out["dB_%d_%d" % (n, k)] = np.array([[bs.dB(th, k, i, t) for i in range(n)] for th in thetas])

    # (iii) compute_control_points
    rng = np.random.default_rng(1234)
    for n in (7, 10):
        for d in (2, 7, 9):
            via = rng.normal(size=(n, d))
            ctrl, t = bs.compute_control_points(via, 3)
            out["ccp_via_%d_%d" % (n, d)] = via
            out["ccp_ctrl_%d_%d" % (n, d)] = ctrl
            out["ccp_t_%d_%d" % (n, d)] = t

    # (iv) config 1: 2-DoF, p=3, 10 linear vias (0,0)->(1,1), 64 candidates
    p, n, D, B, W = 3, 10, 2, 64, 50
    via = np.linspace(0.0, 1.0, n)[:, None] * np.ones((1, D))
    ctrl0, t = bs.compute_control_points(via, p)
    rng = np.random.default_rng(0)
    cand = np.repeat(ctrl0[None], B, axis=0)
    cand[:, p:n - p, :] += rng.normal(0.0, 0.08, size=(B, n - 2 * p, D)) * 1.0
    u = np.array([i / (W - 1) for i in range(W)])
    pts = np.array([[bs.bspline(ui, t, cand[b], p) for ui in u] for b in range(B)])
    chords = np.linalg.norm(pts[:, 1:] - pts[:, :-1], axis=2)
    arc = np.array([sum(float(c) for c in chords[b]) for b in range(B)])
    best = int(np.argmin(arc))  # np.argmin returns the lowest index on ties
    out.update(cfg1_knots=np.asarray(t, np.float64), cfg1_ctrl0=ctrl0, cfg1_ctrl=cand,
               cfg1_u=u, cfg1_pts=pts, cfg1_arc=arc, cfg1_best=np.array([best]),
               cfg1_p=np.array([p]), cfg1_W=np.array([W]))

    # reference unit-test cases (sspp/tests/test_BSplines.py:73-94)
    th = np.linspace(0, 1, 100)
    tl = bs.knot_vector(7, 1)
    out["lin_vals"] = np.array([bs.bspline(x, tl, np.arange(7).reshape(7, 1), 1) for x in th])
    tc = bs.knot_vector(7, 3)
    out["const_vals"] = np.array([bs.bspline(x, tc, np.ones((7, 9)), 3) for x in th])

    # (vi) the reference's robot path pipeline (scripts/main_bspline.py:198-209): 7 via points
    # in 9-D (7 robocrane joints + 2 passive zeros), k = 2, compute_control_points -> ctr_pts,
    # knot_vec.  Its saved bspline_params.npy is a pickled dict that the safe loader refuses
    # (numpy.load(allow_pickle=False)), so the via points here are seeded joint-angle-like values;
    # the knot vector is the one SURVEY §8c recorded from that file.  Outputs: bspline() on the
    # arc-length grid of 128 check points and its arc length.
    rng = np.random.default_rng(2025)
    via = np.zeros((7, 9))
    via[:, :7] = np.cumsum(rng.uniform(-0.35, 0.35, size=(7, 7)), axis=0)
    ctrl, t = bs.compute_control_points(via, 2)
    W = 128
    u = np.array([i / (W - 1) for i in range(W)])
    pts = np.array([bs.bspline(ui, t, ctrl, 2) for ui in u])
    chords = np.linalg.norm(pts[1:] - pts[:-1], axis=1)
    out.update(robot_via=via, robot_ctrl=ctrl, robot_knots=np.asarray(t, np.float64), robot_u=u,
               robot_pts=pts, robot_arc=np.array([sum(float(c) for c in chords)]))

    # (v) CubicPath
    cp = cpm.CubicPath()
    start, viap, end = np.array([0.0, 0.5, 1.0]), np.array([0.7, 1.2, 0.3]), np.array([2.0, 0.0, 0.5])
    cp.plan(start, viap, end)
    uu = np.linspace(-0.1, 1.1, 25)
    res = [cp.evaluate_with_derivatives(x) for x in uu]
    out.update(cubic_start=start, cubic_via=viap, cubic_end=end, cubic_u=uu,
               cubic_pos=np.array([r[0] for r in res]), cubic_vel=np.array([r[1] for r in res]),
               cubic_acc=np.array([r[2] for r in res]))

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, "keys:", len(out))


if __name__ == "__main__":
    main()

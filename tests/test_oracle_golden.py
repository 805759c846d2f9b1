"""Pin the oracle (oracle/sspp_oracle.c) against the reference's own Python vectors and closed forms.

Golden vectors: tests/golden/bsplines_golden.npz, generated from the reference's
sspp/BSplines.py and sspp/CubicPath.py by tests/golden/make_golden.py.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O


def test_knot_vectors_match_reference(golden):
    for n, k in golden["kv_nk"]:
        np.testing.assert_array_equal(O.py_knot_vector(int(n), int(k)), golden["kv_%d_%d" % (n, k)])


@pytest.mark.parametrize("n,k", [(5, 3), (10, 3), (7, 2), (7, 1)])
def test_basis_tables_match_reference(golden, n, k):
    t = O.py_knot_vector(n, k)
    th = golden["basis_theta"]
    got = np.array([[O.lib().or_py_B(float(x), k, i, t) for i in range(n)] for x in th])
    np.testing.assert_array_equal(got, golden["B_%d_%d" % (n, k)])


def test_config1_points_and_arc_lengths(golden):
    """Config 1: de Boor evaluation == BSplines.bspline; arc length + argmin."""
    t, C, u = golden["cfg1_knots"], golden["cfg1_ctrl"], golden["cfg1_u"]
    pts = np.array([[O.spline_eval(t, 3, C[b], x) for x in u] for b in range(C.shape[0])])
    assert np.abs(pts - golden["cfg1_pts"]).max() <= 1e-15
    py = np.array([[O.py_bspline(x, t, C[b], 3) for x in u] for b in range(4)])
    np.testing.assert_array_equal(py, golden["cfg1_pts"][:4])
    for seq in (False, True):
        arc, feas = O.sspp_score(None, t, 3, C, int(golden["cfg1_W"][0]), sequential=seq)
        assert feas.all()
        assert np.abs(arc - golden["cfg1_arc"]).max() <= 1e-14
        assert O.argmin(arc, feas)[0] == int(golden["cfg1_best"][0])


def test_reference_unit_tests_constant_and_linear(golden):
    """sspp/tests/test_BSplines.py:73-94 restated on the oracle."""
    th = np.linspace(0, 1, 100)
    tl = O.py_knot_vector(7, 1)
    lin = np.array([O.py_bspline(x, tl, np.arange(7.0).reshape(7, 1), 1) for x in th])
    np.testing.assert_array_equal(lin, golden["lin_vals"])
    assert np.allclose(lin.ravel(), np.linspace(0, 6, 100), atol=1e-6)
    tc = O.py_knot_vector(7, 3)
    const = np.array([O.py_bspline(x, tc, np.ones((7, 9)), 3) for x in th])
    np.testing.assert_array_equal(const, golden["const_vals"])


def test_knot_averaging_closed_form():
    """Eigen KnotAveraging for u_i = i/9, p = 3: interior knots 2/9 .. 7/9."""
    u = np.array([i / 9 for i in range(10)])
    k = O.knot_averaging(u, 3)
    assert k.shape == (14,)
    np.testing.assert_array_equal(k[:4], 0.0)
    np.testing.assert_array_equal(k[-4:], 1.0)
    np.testing.assert_allclose(k[4:10], np.arange(2, 8) / 9, atol=1e-15)


@pytest.mark.parametrize("n,p,D", [(10, 3, 7), (7, 3, 9), (3, 2, 4), (5, 2, 4), (4, 3, 2)])
def test_interpolation_known_answers(n, p, D):
    """Interpolate: endpoints, via residuals ~1e-15, Greville abscissae for linear data."""
    rng = np.random.default_rng(n * 10 + p)
    u = np.array([i / (n - 1) for i in range(n)])
    pts = rng.normal(size=(n, D))
    knots, ctrl = O.interpolate(pts, p, u)
    for i in range(n):
        assert np.abs(O.spline_eval(knots, p, ctrl, u[i]) - pts[i]).max() <= 1e-12
    np.testing.assert_allclose(ctrl[0], pts[0], rtol=0, atol=1e-14)
    a, b = rng.normal(size=D), rng.normal(size=D)
    lin = np.array([(1 - t) * a + t * b for t in u])
    knots, ctrl = O.interpolate(lin, p, u)
    grev = np.array([knots[j + 1:j + p + 1].mean() for j in range(n)])
    np.testing.assert_allclose(ctrl, a + grev[:, None] * (b - a), atol=1e-13)


def test_tsp_bezier_known_answer():
    """K = 1, p = 2: knots [0,0,0,1,1,1]; middle control point = 2 via - (start + end)/2."""
    s, v, e = np.array([0.2, 0, 0.1, 0]), np.array([0.1, 0.3, 0.4, 0.5]), np.array([0, 0, 0.3, 1])
    knots, ctrl = O.interpolate(np.stack([s, v, e]), 2, np.array([0, 0.5, 1.0]))
    np.testing.assert_array_equal(knots, [0, 0, 0, 1, 1, 1])
    np.testing.assert_allclose(ctrl[1], 2 * v - 0.5 * (s + e), atol=1e-15)


def test_partition_of_unity_and_span():
    u = np.array([i / 9 for i in range(10)])
    knots = O.knot_averaging(u, 3)
    for x in np.random.default_rng(0).uniform(0, 1, 200).tolist() + [0.0, 1.0, 2 / 9, 7 / 9]:
        N = O.basis(x, 3, knots)
        assert abs(N.sum() - 1.0) <= 1e-15
        assert (N >= -1e-16).all()
    assert O.span(0.0, 3, knots) == 3
    assert O.span(1.0, 3, knots) == 9  # n - 1


def test_canonical_sum():
    x = np.arange(1.0, 128.0)  # exact in binary
    assert O.canon_sum(x) == x.sum()
    r = np.random.default_rng(1).normal(size=255)
    assert abs(O.canon_sum(r) - np.sum(r)) <= 1e-13
    assert O.lib().or_lanes_for(127) == 128
    assert O.lib().or_lanes_for(255) == 256
    assert O.lib().or_lanes_for(2000) == 256
    assert O.lib().or_lanes_for(1) == 64


def test_philox_known_answer():
    """Random123 Philox4x32-10 known-answer vectors (kat_vectors)."""
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xffffffff] * 4, [0xffffffff] * 2) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6,
                                                            0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                    [0xa4093822, 0x299f31d0]) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_normal_sampler_statistics():
    """FP64 Box-Muller pairs (the default sampler of both planners): moments, tails, pairing."""
    z = np.array([O.normal_pair(7, g, m, 0) for g in range(20000) for m in range(2)]).ravel()
    assert abs(z.mean()) < 0.01
    assert abs(z.std() - 1.0) < 0.01
    assert abs(np.mean(z ** 4) - 3.0) < 0.1
    for q, x in ((0.5, 0.0), (0.8413, 1.0), (0.9772, 2.0), (0.99865, 3.0)):
        assert abs((z < x).mean() - q) < 0.01
    assert abs(np.corrcoef(z[0::2], z[1::2])[0, 1]) < 0.02


def test_normal_pair64_accuracy():
    """The written-out FP64 ln / sincos polynomials of the default sampler agree with libm to a
    few ulp over 200k normals (std::normal_distribution<double> precision class), the maximum
    |z| is reachable (u1 = 2^-53 -> sqrt(-2 ln 2^-53) = 8.5717) and u1 = 1 gives exactly 0."""
    worst = 0.0
    for g in range(50000):
        for m in range(2):
            a = np.array(O.normal_pair(3, g, m, 0))
            b = np.array(O.normal_pair(3, g, m, 0, libm=True))
            worst = max(worst, float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3))))
    assert worst < 2e-15, worst
    import ctypes as C
    lib = O.lib()
    lib.or_bm_log64_test.restype = C.c_double
    lib.or_bm_log64_test.argtypes = [C.c_double]
    for u in (2.0 ** -53, 1e-9, 0.3, 0.70710678118654757, 0.7071067811865476, 0.5, 0.999999, 1.0):
        assert abs(lib.or_bm_log64_test(u) - np.log(u)) <= 2.5e-16 * max(1.0, abs(np.log(u)))
    assert lib.or_bm_log64_test(1.0) == 0.0
    assert abs(np.sqrt(-2.0 * lib.or_bm_log64_test(2.0 ** -53)) - 8.5717) < 1e-4


def test_normal_quad_statistics():
    """FP32 Box-Muller quads (SamplingPathPlanner sampler): moments, tails and the pairing."""
    z = np.array([O.normal_quad(11, g, m, 0) for g in range(20000) for m in range(2)]).ravel()
    assert abs(z.mean()) < 0.01
    assert abs(z.std() - 1.0) < 0.01
    assert abs(np.mean(z ** 4) - 3.0) < 0.1  # Gaussian kurtosis
    assert 5.0 < np.abs(z).max() < 5.8       # u1 >= 2^-24: |z| <= sqrt(-2 ln 2^-24) = 5.77
    for q in (0.5, 0.8413, 0.9772):          # CDF at 0, 1, 2 sigma
        x = {0.5: 0.0, 0.8413: 1.0, 0.9772: 2.0}[q]
        assert abs((z < x).mean() - q) < 0.01
    assert abs(np.corrcoef(z[0::4], z[1::4])[0, 1]) < 0.02


def test_sample_sspp_rule():
    """sampleWithNoise perturbs only columns j in [p, n-p) (include/sspp.h:121-127)."""
    init = np.arange(70.0).reshape(10, 7)
    out = O.sample_sspp(init, 3, 0.1, np.linspace(1, 2, 7), 1, 0, 5)
    np.testing.assert_array_equal(out[:, :3], np.broadcast_to(init[:3], (5, 3, 7)))
    np.testing.assert_array_equal(out[:, 7:], np.broadcast_to(init[7:], (5, 3, 7)))
    assert (out[:, 3:7] != init[3:7]).all()
    again = O.sample_sspp(init, 3, 0.1, np.linspace(1, 2, 7), 1, 2, 3)
    np.testing.assert_array_equal(again, out[2:5])  # counter-based: ids, not call order


def test_sample_tsp_rules():
    """Sampler::sample: truncated normal xyz in [lo, hi], wrapped yaw, z >= z_min."""
    mean = np.array([[0.0, 0.0, 0.05, 1.5]])
    sig = np.array([[0.5, 0.01, 0.3, 0.5]])
    lo, hi = np.array([-0.1, -1, 0.0, -1.6]), np.array([0.1, 1, 0.6, 1.6])
    v = O.sample_tsp(mean, sig, lo, hi, 0.02, 3, 0, 4000)[:, 0]
    assert (v[:, 0] >= -0.1).all() and (v[:, 0] <= 0.1).all()
    assert (v[:, 2] >= 0.02).all()
    assert (v[:, 3] >= -1.6).all() and (v[:, 3] <= 1.6).all()
    assert (v[:, 3] < 0).any()  # wrapped around
    fixed = O.sample_tsp(mean, sig, np.array([-1, -1, 0, 0.3]), np.array([1, 1, 1, 0.3]), 0, 3, 0, 10)
    np.testing.assert_array_equal(fixed[:, 0, 3], 1.5)  # lo == hi: yaw = mean


def test_robot_path_d9_p2_golden(golden):
    """Degree-2, 9-D robot path of the reference's main_bspline.py pipeline: the oracle's spline
    evaluation (A2.1/A2.2 basis) reproduces the reference bspline() points and arc length."""
    knots, ctrl, u = golden["robot_knots"], golden["robot_ctrl"], golden["robot_u"]
    pts = np.array([O.spline_eval(knots, 2, ctrl, x) for x in u])
    assert np.abs(pts - golden["robot_pts"]).max() <= 1e-13
    arc, _ = O.sspp_score(None, knots, 2, ctrl[None], 128)
    assert abs(arc[0] - golden["robot_arc"][0]) <= 1e-12


def test_reference_robot_path_fixture():
    """The reference's saved robot path (scripts/bspline_params.npy, main_bspline.py:198-209;
    tests/golden/make_robot_path.py): 7 joint angles + 2 passive joints, degree 2, knots
    [0,0,0,.2,.4,.6,.8,1,1,1].  The oracle's spline evaluation equals the reference's
    BSplines.bspline on 128 points and its computeArcLength the chord sum over them."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "robot_path.json")))
    knots, ctrl, k = np.array(d["knots"]), np.array(d["ctrl"]), d["k"]
    assert ctrl.shape == (7, 9) and k == 2
    pts = np.array([O.spline_eval(knots, k, ctrl, u) for u in d["u"]])
    assert np.abs(pts - np.array(d["bspline"])).max() <= 1e-13
    arc, feas = O.sspp_score(None, knots, k, ctrl[None], d["W"])
    assert feas[0] == 1 and abs(arc[0] - d["arc_length"]) <= 1e-12


def test_log_table():
    """The FP64 sampler's ln table (sspp_amd/csrc/sspp_logtab.h, shared data of the kernels and the
    oracle), recomputed here independently: entry k - 64 holds r = RN(64 / k) and -ln r as
    hi + lo, hi the double nearest -ln r and lo the double nearest the remainder (40-digit
    decimal logarithms); the table's hex literals are parsed from the header text."""
    import os
    import re
    from decimal import Decimal, getcontext
    getcontext().prec = 40
    path = os.path.join(os.path.dirname(__file__), "..", "sspp_amd", "csrc", "sspp_logtab.h")
    rows = re.findall(r"\{(0x[^}]*)\}", open(path).read())
    assert len(rows) == 64
    for k, row in zip(range(64, 128), rows):
        r, hi, lo, pad = (float.fromhex(x.strip()) for x in row.split(","))
        assert r == 64.0 / k and pad == 0.0
        L = -Decimal(r).ln()
        assert hi == float(L)
        assert lo == float(L - Decimal(hi))
        assert abs(Decimal(hi) + Decimal(lo) - L) < Decimal(2) ** -105

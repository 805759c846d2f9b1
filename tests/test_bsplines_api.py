"""`from sspp import BSplines, CubicPath` — same API and values as the reference's modules.

Includes the reference's own suite (sspp/tests/test_BSplines.py) restated against the drop-in.
"""
import numpy as np
import pytest

from sspp import BSplines as bs
from sspp import CubicPath as cpm


@pytest.mark.parametrize("n,k", [(5, 3), (10, 3), (7, 2), (7, 1)])
def test_basis_and_derivative_bitwise(golden, n, k):
    t = bs.knot_vector(n, k)
    th = golden["basis_theta"]
    np.testing.assert_array_equal([[bs.B(x, k, i, t) for i in range(n)] for x in th], golden["B_%d_%d" % (n, k)])
    np.testing.assert_array_equal([[bs.dB(x, k, i, t) for i in range(n)] for x in th], golden["dB_%d_%d" % (n, k)])


def test_knot_vector_and_control_points(golden):
    for n, k in golden["kv_nk"]:
        np.testing.assert_array_equal(bs.knot_vector(int(n), int(k)), golden["kv_%d_%d" % (n, k)])
    for n in (7, 10):
        for d in (2, 7, 9):
            c, t = bs.compute_control_points(golden["ccp_via_%d_%d" % (n, d)], 3)
            np.testing.assert_array_equal(c, golden["ccp_ctrl_%d_%d" % (n, d)])
            np.testing.assert_array_equal(t, golden["ccp_t_%d_%d" % (n, d)])


def test_bspline_values_and_edges(golden):
    t, C, u = golden["cfg1_knots"], golden["cfg1_ctrl"], golden["cfg1_u"]
    np.testing.assert_array_equal([[bs.bspline(x, t, C[b], 3) for x in u] for b in range(8)],
                                  golden["cfg1_pts"][:8])
    c = C[0]
    np.testing.assert_array_equal(bs.bspline(1.0, t, c, 3), c[-1])           # theta >= 1
    np.testing.assert_array_equal(bs.bspline(-0.5, t, c, 3), c[0] * 1.0)     # theta < 0
    assert sum(bs.B(1.0, 3, i, t) for i in range(10)) == 0.0                  # half-open (Q12)


def test_cubic_path(golden):
    cp = cpm.CubicPath()
    assert cp.plan(golden["cubic_start"], golden["cubic_via"], golden["cubic_end"])
    for i, x in enumerate(golden["cubic_u"]):
        p, v, a = cp.evaluate_with_derivatives(x)
        np.testing.assert_array_equal(p, golden["cubic_pos"][i])
        np.testing.assert_array_equal(v, golden["cubic_vel"][i])
        np.testing.assert_array_equal(a, golden["cubic_acc"][i])
        np.testing.assert_array_equal(cp.evaluate(x), golden["cubic_pos"][i])
    np.testing.assert_allclose(cp.evaluate(0.5), golden["cubic_via"], atol=1e-15)


# ---- the reference's unit tests (sspp/tests/test_BSplines.py), restated --------------------
K, N = 3, 5
T = bs.knot_vector(N, K)
CC = np.array([0, 1, 2, 3, 4])


def test_ref_basis_properties():
    r = bs.B(0.5, K, 2, T)
    assert isinstance(r, float) and 0.0 <= r <= 1.0


def test_ref_types():
    assert isinstance(bs.dB(0.5, K, 2, T), float)
    assert isinstance(bs.bspline(0.5, T, CC, K), float)
    assert isinstance(bs.bspline_derivative(0.5, T, CC, K), float)


def test_ref_knot_vector():
    t = bs.knot_vector(N, K)
    assert len(t) == N + K + 1
    assert np.all(t[:K] == 0) and np.all(t[-K:] == 1)


def test_ref_control_points_shape():
    via = np.array([[0, 0], [1, 2], [2, 3], [3, 5], [4, 6]])
    c, t = bs.compute_control_points(via, K)
    assert c.shape == via.shape and len(t) == len(T)


def test_ref_constant_and_linear():
    th = np.linspace(0, 1, 100)
    y = np.array([bs.bspline(x, bs.knot_vector(7, 3), np.ones((7, 9)), 3) for x in th])
    assert np.allclose(y, 1)
    y = np.array([bs.bspline(x, bs.knot_vector(7, 1), np.arange(7).reshape(7, 1), 1) for x in th])
    assert np.allclose(y, np.linspace(0, 6, 100).reshape(100, 1), atol=1e-6)

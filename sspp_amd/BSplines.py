"""B-spline operator API — drop-in for the reference's ``sspp/BSplines.py`` (NumPy part).

Same names, arguments, return types and edge behaviour as the reference
(/root/reference/sspp/BSplines.py):

  B(theta, k, i, t)                  Cox–de Boor basis, half-open support (line 11-29; SURVEY Q12:
                                     every basis is 0 at theta == 1)
  dB(theta, k, i, t)                 basis derivative (31-42)
  bspline(theta, t, c, k)            theta < 0 -> c[0] * B(0, k, 0, t); theta >= 1 -> c[n-1] (44-51)
  bspline_derivative(theta, t, c, k) (53-55)
  knot_vector(n_control_points, k)   k zeros + linspace(0, 1, n+1-k) + k ones (58-62)
  compute_control_points(via, k)     collocation at theta_i = i/(n-1), A[0,0]=A[n-1,n-1]=1,
                                     least squares (65-106) -> (control_points, t)
  evalRotationInterpolation*(...)    SLERP helpers (114-132)

Implementation is independent of the reference: the basis is built bottom-up (degree 0 ->
k) over the k+1 supporting knot spans, with the same per-term arithmetic as the recursive
definition, so values agree with the reference bit for bit.  CasADi symbolic twins
(casadiBspline & co., 138-208) need CasADi, which is not part of the scoring path; they raise
ImportError when CasADi is absent.

For batched scoring on the GPU use ``sspp_amd.SsppJob`` (``sample_score`` / ``score_ctrl``)
or the drop-in ``from sspp import _sspp`` planner.
"""
from __future__ import annotations

import numpy as np


def _basis_table(theta, k, i, t):
    """N[j] = B(theta, d, i + j, t) for the current degree d, starting at d = 0."""
    N = [1.0 if t[i + j] <= theta < t[i + j + 1] else 0.0 for j in range(k + 1)]
    for d in range(1, k + 1):
        nxt = []
        for j in range(k + 1 - d):
            a = i + j
            if t[a + d] == t[a]:
                left = 0.0
            else:
                left = (theta - t[a]) / (t[a + d] - t[a]) * N[j]
            if t[a + d + 1] == t[a + 1]:
                right = 0.0
            else:
                right = (t[a + d + 1] - theta) / (t[a + d + 1] - t[a + 1]) * N[j + 1]
            nxt.append(left + right)
        N = nxt
    return N


def B(theta, k, i, t):
    """Value of the i-th B-spline basis function of degree k at theta."""
    return _basis_table(theta, k, i, t)[0]


def dB(theta, k, i, t):
    """Derivative of the i-th degree-k basis function at theta."""
    if k == 0:
        return 0.0
    lo = 0.0 if t[i + k] == t[i] else k / (t[i + k] - t[i]) * B(theta, k - 1, i, t)
    hi = 0.0 if t[i + k + 1] == t[i + 1] else -k / (t[i + k + 1] - t[i + 1]) * B(theta, k - 1, i + 1, t)
    return lo + hi


def bspline(theta, t, c, k):
    """Evaluate sum_i c[i] * B_i(theta) (c: (n,) or (n, d))."""
    n = len(t) - k - 1
    if theta < 0:
        return c[0] * B(0, k, 0, t)
    if theta >= 1:
        return c[n - 1]
    acc = 0
    for i in range(n):
        acc = acc + c[i] * B(theta, k, i, t)
    return acc


def bspline_derivative(theta, t, c, k):
    n = len(t) - k - 1
    acc = 0
    for i in range(n):
        acc = acc + c[i] * dB(theta, k, i, t)
    return acc


def knot_vector(n_control_points, k):
    """Clamped uniform knot vector with n_control_points + k + 1 entries."""
    inner = np.linspace(0, 1, n_control_points + 1 - k)
    return np.concatenate(([0] * k, inner, [1] * k))


def compute_control_points(via_points, k):
    """Control points whose spline passes (in the least-squares sense) through via_points.

    Returns (control_points (n, d), knot vector t).
    """
    via_points = np.asarray(via_points)
    n = len(via_points)
    t = knot_vector(n, k)
    A = np.zeros((n, n))
    for row in range(n):
        theta = row / (n - 1)
        for col in range(n):
            A[row, col] = B(theta, k, col, t)
    A[0, 0] = 1.0
    A[n - 1, n - 1] = 1.0
    ctrl = np.linalg.lstsq(A, via_points, rcond=None)[0]
    return ctrl, t


# ------------------------------------------------------------------ SLERP helpers
def evalRotationInterpolation(R0, theta, S, phi):
    """Rodrigues interpolation R0 (I + sin(theta phi) S + (1 - cos(theta phi)) S^2)."""
    a = theta * phi
    return np.dot(R0, np.eye(3) + np.sin(a) * S + (1 - np.cos(a)) * np.dot(S, S))


def evalRotationInterpolationDiff(R0, theta, S, phi):
    a = theta * phi
    return np.dot(R0, np.cos(a) * S + np.sin(a) * np.dot(S, S))


def _segment(theta, theta_vec):
    for seg in range(len(theta_vec) - 1):
        if theta_vec[seg] <= theta < theta_vec[seg + 1]:
            return seg
    return None


def evalRotationInterpolationFull(R, phi, S, theta, theta_vec):
    seg = _segment(theta, theta_vec)
    if seg is None:
        return None
    s = (theta - theta_vec[seg]) / (theta_vec[seg + 1] - theta_vec[seg])
    return evalRotationInterpolation(R[seg], s, S[seg], phi[seg])


def evalRotationInterpolationDiffFull(R, phi, S, theta, theta_vec):
    seg = _segment(theta, theta_vec)
    if seg is None:
        return None
    s = (theta - theta_vec[seg]) / (theta_vec[seg + 1] - theta_vec[seg])
    return evalRotationInterpolationDiff(R[seg], s, S[seg], phi[seg])


def _casadi():
    try:
        import casadi  # noqa: F401
    except ImportError as e:  # pragma: no cover - casadi is not in this image
        raise ImportError("the CasADi symbolic B-spline twins need casadi; the NumPy API and the "
                          "GPU scorer do not") from e
    return casadi


def casadiBspline(theta, t, c, k):  # pragma: no cover - symbolic, needs casadi
    ca = _casadi()
    n = t.shape[0] - k - 1
    return sum(c[i] * casadiB(theta, k, i, t) for i in range(n)) if n else ca.MX(0)


def casadiB(theta, k, i, t):  # pragma: no cover - symbolic, needs casadi
    ca = _casadi()
    if k == 0:
        return ca.if_else(ca.logic_and(t[i] <= theta, theta < t[i + 1]), 1.0, 0.0)
    lo = 0.0 if t[i + k] == t[i] else (theta - t[i]) / (t[i + k] - t[i]) * casadiB(theta, k - 1, i, t)
    hi = 0.0 if t[i + k + 1] == t[i + 1] else (t[i + k + 1] - theta) / (t[i + k + 1] - t[i + 1]) * \
        casadiB(theta, k - 1, i + 1, t)
    return lo + hi


__all__ = ["B", "dB", "bspline", "bspline_derivative", "knot_vector", "compute_control_points",
           "evalRotationInterpolation", "evalRotationInterpolationDiff",
           "evalRotationInterpolationFull", "evalRotationInterpolationDiffFull", "casadiBspline",
           "casadiB"]

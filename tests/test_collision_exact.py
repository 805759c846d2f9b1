"""Exactness of the cylinder-box narrowphase and the box-box contact manifold.

MuJoCo is absent here, so the restated collision rules are pinned by independent
geometry, not by MuJoCo output:

* cylinder-box: the signed distance of two convex bodies is max over unit directions n of their
  separation along n.  The reference below evaluates that separation (from the support
  functions) on a dense Fibonacci sphere and refines the best directions by a shrinking random
  search — no candidate-axis reasoning at all — and the oracle's contact (dist < margin) and
  deep-contact (dist < -1e-3, include/Collision.h:93) decisions must agree with it on random
  oriented pairs, near-threshold cases skipped.
* box-box: SAT is exact for boxes; the manifold's deep count is checked on hand configurations
  with known contact polygons and on random pairs (>= 1 exactly when the SAT depth > 1e-3).
"""
import math

import numpy as np
import pytest

from tests.test_collision_known import BOX, CYL, _qmat, contacts

DEEP = -1e-3


def _fib_sphere(n):
    i = np.arange(n) + 0.5
    phi = np.arccos(1 - 2 * i / n)
    th = math.pi * (1 + 5 ** 0.5) * i
    return np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1)


def _sep(ns, T, a, H, R, Bm, e):
    """separation along unit directions ns (M, 3): |T.n| - (h_cyl(n) + h_box(n))"""
    an = ns @ a
    perp = np.sqrt(np.maximum(1.0 - an * an, 0.0))
    return np.abs(ns @ T) - (H * np.abs(an) + R * perp + np.abs(ns @ Bm) @ e)


def ref_signed_distance(T, a, H, R, Bm, e, rng, dense=40000, rounds=60):
    """max over the sphere of the separation: dense sampling + shrinking random refinement"""
    ns = _fib_sphere(dense)
    s = _sep(ns, T, a, H, R, Bm, e)
    top = np.argsort(-s)[:8]
    best_n, best = ns[top], s[top]
    scale = 0.05
    for _ in range(rounds):
        cand = best_n[:, None, :] + scale * rng.normal(size=(len(best_n), 48, 3))
        cand /= np.linalg.norm(cand, axis=2, keepdims=True)
        cs = _sep(cand.reshape(-1, 3), T, a, H, R, Bm, e).reshape(len(best_n), -1)
        k = cs.argmax(1)
        better = cs[np.arange(len(best_n)), k] > best
        best_n[better] = cand[better, k[better]]
        best[better] = cs[better, k[better]]
        scale *= 0.75
    return best.max()


def sat7_lower_bound(T, a, H, R, Bm, e):
    """the 7 finite SAT axes alone (round-1 restatement): a lower bound of the distance"""
    axes = [Bm[:, k] for k in range(3)] + [a] + [np.cross(a, Bm[:, k]) for k in range(3)]
    axes = np.array([x / np.linalg.norm(x) for x in axes if np.linalg.norm(x) > 1e-9])
    return _sep(axes, T, a, H, R, Bm, e).max()


def _random_pair(rng):
    R, H = rng.uniform(0.02, 0.15), rng.uniform(0.02, 0.15)
    e = rng.uniform(0.02, 0.2, 3)
    qc, qb = rng.normal(size=4), rng.normal(size=4)
    qc, qb = qc / np.linalg.norm(qc), qb / np.linalg.norm(qb)
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    # centre distance spread around touching (reach along d of both bodies)
    reach = np.linalg.norm(e) + math.hypot(R, H)
    T = d * rng.uniform(0.3, 1.05) * reach
    return R, H, e, qc, qb, T


@pytest.mark.parametrize("margin", [0.0, 0.001, 0.01])
def test_cylinder_box_contact_matches_support_function_reference(margin):
    rng = np.random.default_rng(7 + int(margin * 1000))
    n, agree, sat7_wrong, deep_checked = 0, 0, 0, 0
    for _ in range(450):
        R, H, e, qc, qb, T = _random_pair(rng)
        Mc, Mb = _qmat(qc), _qmat(qb)
        a = Mc[:, 2]
        dist = ref_signed_distance(T, a, H, R, Mb, e, rng)
        cont, cost, nd = contacts([(CYL, (R, H, 0), (0, 0, 0), tuple(qc), margin)],
                                  [(BOX, tuple(e), (0, 0, 0), (1, 0, 0, 0))], T, tuple(qb))
        if abs(dist - margin) > 1e-6:
            n += 1
            agree += (cont > 0) == (dist < margin)
            sat7_wrong += (sat7_lower_bound(T, a, H, R, Mb, e) < margin) != (dist < margin)
        if abs(dist - DEEP) > 1e-6:
            deep_checked += 1
            assert (nd > 0) == (dist < DEEP), (R, H, e, qc, qb, T, dist)
    assert n > 400 and agree == n
    assert deep_checked > 400
    # the configurations exercise the non-SAT families: the 7-axis test alone errs on some
    assert sat7_wrong > 0


@pytest.mark.parametrize("margin", [0.0, 0.001, 0.01])
def test_upright_cylinder_box_matches_support_function_reference(margin):
    """Vertical cylinder vs upright box (both turned about z only, as a yaw-only TaskSpacePlanner
    mover keeps them): the oracle takes the prism formula (cb_upright_sd, the device's
    sspd::cb_upright_sd); its contact and deep decisions must agree with the same independent
    support-function reference, stacked, side-by-side and corner configurations alike."""
    rng = np.random.default_rng(70 + int(margin * 1000))
    n, deep_checked = 0, 0
    for it in range(450):
        R, H = rng.uniform(0.02, 0.15), rng.uniform(0.02, 0.15)
        e = rng.uniform(0.02, 0.2, 3)
        yc, yb = rng.uniform(-math.pi, math.pi, 2)
        qc = (math.cos(yc / 2), 0.0, 0.0, math.sin(yc / 2))
        qb = (math.cos(yb / 2), 0.0, 0.0, math.sin(yb / 2))
        if it % 3 == 0:  # on top of the box / below it
            T = np.array([rng.uniform(-1, 1) * (e[0] + R), rng.uniform(-1, 1) * (e[1] + R),
                          rng.choice([-1, 1]) * (e[2] + H) * rng.uniform(0.9, 1.05)])
        else:
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            T = d * rng.uniform(0.3, 1.05) * (np.linalg.norm(e) + math.hypot(R, H))
        Mc, Mb = _qmat(qc), _qmat(qb)
        dist = ref_signed_distance(T, Mc[:, 2], H, R, Mb, e, rng)
        cont, cost, nd = contacts([(CYL, (R, H, 0), (0, 0, 0), qc, margin)],
                                  [(BOX, tuple(e), (0, 0, 0), (1, 0, 0, 0))], T, qb)
        if abs(dist - margin) > 1e-6:
            n += 1
            assert (cont > 0) == (dist < margin), (R, H, e, qc, qb, T, dist)
        if abs(dist - DEEP) > 1e-6:
            deep_checked += 1
            assert (nd > 0) == (dist < DEEP), (R, H, e, qc, qb, T, dist)
    assert n > 400 and deep_checked > 400


# ---------------------------------------------------------------- box-box manifold
BIG = (BOX, (0.3, 0.3, 0.1), (0, 0, 0), (1, 0, 0, 0))


def _deep(moving_size, pos, quat=(1, 0, 0, 0), static=BIG):
    return contacts([static], [(BOX, moving_size, (0, 0, 0), (1, 0, 0, 0))], pos, quat)


def test_box_box_manifold_face_contacts():
    # a 45-degree-rotated small box sunk 5 mm into the big box's top face: 4 corners inside
    q45 = (math.cos(math.pi / 8), 0, 0, math.sin(math.pi / 8))
    assert _deep((0.05, 0.05, 0.05), (0, 0, 0.145), q45)[2] == 4
    # sunk only 0.5 mm: in contact, no deep contact
    n, _, nd = _deep((0.05, 0.05, 0.05), (0, 0, 0.1495), q45)
    assert (n, nd) == (1, 0)
    # equal footprints, offset by half a box in y: two incident corners + two clip points
    eq = (BOX, (0.1, 0.1, 0.1), (0, 0, 0), (1, 0, 0, 0))
    assert _deep((0.1, 0.1, 0.1), (0, 0.1, 0.195), static=eq)[2] == 4
    # partly overhanging the big box's edge: corners outside are clipped to the side plane
    assert _deep((0.05, 0.05, 0.05), (0.28, 0, 0.145))[2] == 4


def test_box_box_manifold_tilted_edge_and_edge_edge():
    # tilted about x so that one bottom edge dips 5 mm deep and the other is above the face
    ang = 0.2
    qx = (math.cos(ang / 2), math.sin(ang / 2), 0, 0)
    e = 0.05
    low = e * math.cos(ang) + e * math.sin(ang)  # depth of the lowest edge below the centre
    n, _, nd = _deep((e, e, e), (0, 0, 0.1 + low - 0.005), qx)
    assert nd == 2
    # edge against edge: two boxes rotated 45 deg about orthogonal horizontal axes
    s = math.sqrt(2) * 0.05
    qa = (math.cos(math.pi / 8), math.sin(math.pi / 8), 0, 0)
    qb = (math.cos(math.pi / 8), 0, math.sin(math.pi / 8), 0)
    a = (BOX, (0.05, 0.05, 0.05), (0, 0, 0), qa)
    n, _, nd = contacts([a], [(BOX, (0.05, 0.05, 0.05), (0, 0, 0), (1, 0, 0, 0))], (0, 0, 2 * s - 0.004), qb)
    assert (n, nd) == (1, 1)
    n, _, nd = contacts([a], [(BOX, (0.05, 0.05, 0.05), (0, 0, 0), (1, 0, 0, 0))], (0, 0, 2 * s - 0.0005), qb)
    assert (n, nd) == (1, 0)


def _clip_convex(P, Q):
    """Sutherland-Hodgman: convex polygon P (CCW, k x 2) clipped to convex polygon Q (CCW)."""
    out = [np.asarray(p, float) for p in P]
    for i in range(len(Q)):
        a, b = np.asarray(Q[i], float), np.asarray(Q[(i + 1) % len(Q)], float)
        side = lambda p: (b[0] - a[0]) * (p[1] - a[1]) - (b[1] - a[1]) * (p[0] - a[0])  # noqa: E731
        inp, out = out, []
        for j in range(len(inp)):
            cur, nxt = inp[j], inp[(j + 1) % len(inp)]
            sc, sn = side(cur), side(nxt)
            if sc >= 0:
                out.append(cur)
            if (sc >= 0) != (sn >= 0):
                out.append(cur + (nxt - cur) * (sc / (sc - sn)))
    return out


def _rect(cx, cy, a, b, yaw):
    c, s = math.cos(yaw), math.sin(yaw)
    return [(cx + c * x - s * y, cy + s * x + c * y) for x, y in ((-a, -b), (a, -b), (a, b), (-a, b))]


def test_box_box_manifold_non_square_overlap():
    """Face-on-face contacts whose overlap is not the incident face itself: a thin rectangle,
    yawed, sunk 5 mm into the big box's top face across the face's edge.  Every clipped point
    is 5 mm deep, so the deep count is the number of vertices of the exact intersection of the
    two rectangles (computed independently here by polygon clipping)."""
    q = lambda yaw: (math.cos(yaw / 2), 0, 0, math.sin(yaw / 2))  # noqa: E731
    # yawed 30 deg, one corner past x = 0.3: three corners + two points on the edge
    assert _deep((0.1, 0.02, 0.05), (0.21, 0, 0.145), q(math.pi / 6))[2] == 5
    # the big face's corner (0.3, 0.3) inside the rectangle: that corner, the points where the
    # rectangle's edges cross x = 0.3 and y = 0.3, and the rectangle's two corners inside the face
    ref = _rect(0, 0, 0.3, 0.3, 0.0)
    inc = _rect(0.27, 0.27, 0.1, 0.05, math.pi / 4)
    want = len(_clip_convex(inc, ref))
    assert want == 5
    assert _deep((0.1, 0.05, 0.05), (0.27, 0.27, 0.145), q(math.pi / 4))[2] == want
    rng = np.random.default_rng(5)
    seen = set()
    for _ in range(300):
        a, b = rng.uniform(0.02, 0.15), rng.uniform(0.01, 0.15)
        yaw = rng.uniform(-math.pi, math.pi)
        cx, cy = rng.uniform(0.15, 0.29, 2) * rng.choice([-1, 1], 2)
        inc = _rect(cx, cy, a, b, yaw)
        # skip near-degenerate placements (a corner within 1e-6 of the face's edge lines)
        if min(abs(abs(c) - 0.3) for p in inc for c in p) < 1e-6:
            continue
        want = len(_clip_convex(inc, ref))
        assert _deep((a, b, 0.05), (cx, cy, 0.145), q(yaw))[2] == want, (a, b, yaw, cx, cy)
        seen.add(want)
    assert {4, 5, 6} <= seen


def _box_sat_distance(pa, Ma, ea, pb, Mb, eb):
    """exact signed distance of two boxes: max separation over the 15 SAT axes"""
    axes = [Ma[:, i] for i in range(3)] + [Mb[:, j] for j in range(3)]
    axes += [np.cross(Ma[:, i], Mb[:, j]) for i in range(3) for j in range(3)]
    best = -np.inf
    T = pb - pa
    for L in axes:
        n = np.linalg.norm(L)
        if n < 1e-6:
            continue
        L = L / n
        best = max(best, abs(T @ L) - (np.abs(Ma.T @ L) @ ea + np.abs(Mb.T @ L) @ eb))
    return best


def test_box_box_manifold_random_pairs():
    rng = np.random.default_rng(11)
    checked, multi = 0, 0
    for _ in range(400):
        ea, eb = rng.uniform(0.03, 0.2, 3), rng.uniform(0.03, 0.2, 3)
        qa, qb = rng.normal(size=4), rng.normal(size=4)
        qa, qb = qa / np.linalg.norm(qa), qb / np.linalg.norm(qb)
        d = rng.normal(size=3)
        pb = d / np.linalg.norm(d) * rng.uniform(0.3, 1.0) * (np.linalg.norm(ea) + np.linalg.norm(eb))
        dist = _box_sat_distance(np.zeros(3), _qmat(qa), ea, pb, _qmat(qb), eb)
        n, _, nd = contacts([(BOX, ea, (0, 0, 0), qa)], [(BOX, eb, (0, 0, 0), (1, 0, 0, 0))], pb, qb)
        assert 0 <= nd <= 8
        if abs(dist - DEEP) > 1e-9:
            checked += 1
            assert (nd > 0) == (dist < DEEP)
        multi += nd > 1
    assert checked > 390 and multi > 20


def _mat_to_quat(M):
    """rotation matrix (columns = body axes) -> quaternion (w, x, y, z)"""
    tr = np.trace(M)
    if tr > 0:
        s = 2 * math.sqrt(1 + tr)
        return np.array([s / 4, (M[2, 1] - M[1, 2]) / s, (M[0, 2] - M[2, 0]) / s, (M[1, 0] - M[0, 1]) / s])
    i = int(np.argmax(np.diag(M)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = 2 * math.sqrt(1 + M[i, i] - M[j, j] - M[k, k])
    q = np.zeros(4)
    q[0] = (M[k, j] - M[j, k]) / s
    q[1 + i] = s / 4
    q[1 + j] = (M[j, i] + M[i, j]) / s
    q[1 + k] = (M[k, i] + M[i, k]) / s
    return q


def test_cylinder_box_rim_edge_family():
    """A box edge placed at a prescribed gap from the rim along their common normal (built
    directly: a rim point p, a normal n in the rim's normal cone, an edge direction e perpendicular
    to n, the box's two faces at that edge opening away from the cylinder).  The signed distance
    is the gap, so contact (margin 1 mm) and deep contact flip exactly at the thresholds — this
    exercises the rim-edge (ellipse) candidates, which the finite SAT axes do not contain."""
    rng = np.random.default_rng(5)
    R, H = 0.05, 0.04
    margin = 0.001
    checked = flips = 0
    for _ in range(120):
        th = rng.uniform(0, 2 * math.pi)
        s = rng.choice([-1.0, 1.0])
        rho = np.array([math.cos(th), math.sin(th), 0.0])
        p = rho * R + np.array([0, 0, s * H])
        al = rng.uniform(0.15, 1.4)  # normal between the radial direction and the cap normal
        n = math.cos(al) * rho + math.sin(al) * np.array([0, 0, s])
        e = np.cross(n, rng.normal(size=3))
        e /= np.linalg.norm(e)
        w = np.cross(e, n)
        f1, f2 = (-n + w) / math.sqrt(2), (-n - w) / math.sqrt(2)  # outward normals at the edge
        M = np.stack([e, f1, f2], 1)
        ext = np.array([0.08, 0.05, 0.05])
        for gap in (margin + 2e-6, margin - 2e-6, -1e-3 * rng.uniform(0.5, 3.0)):
            q = p + gap * n
            cb = q - ext[1] * f1 - ext[2] * f2
            n_c, _, nd = contacts([(CYL, (R, H, 0), (0, 0, 0), (1, 0, 0, 0), margin)],
                                  [(BOX, tuple(ext), (0, 0, 0), (1, 0, 0, 0))], cb, tuple(_mat_to_quat(M)))
            T, a = cb, np.array([0, 0, 1.0])
            if gap > 0:
                # separated: the closest points are p and q, the distance is the gap
                assert (n_c > 0) == (gap < margin), (th, s, al, gap)
                # the 7 SAT axes alone would not have separated (a false contact)
                flips += sat7_lower_bound(T, a, H, R, M, ext) < margin
            else:
                # penetrating: the depth can be below |gap| (another direction may be shorter)
                dist = ref_signed_distance(T, a, H, R, M, ext, rng)
                assert n_c > 0
                if abs(dist - DEEP) > 1e-6:
                    assert (nd > 0) == (dist < DEEP), (th, s, al, gap, dist)
            checked += 1
    assert checked == 360 and flips > 30

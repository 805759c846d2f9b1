"""Known answers for the collision restatement (oracle/sspp_oracle.c).

MuJoCo is absent, so contact semantics are pinned by hand-computed configurations and, for
box-box intersection, by an independent exact test: two boxes intersect iff the linear program
{x : |A^T (x - a)| <= ea, |B^T (x - b)| <= eb} is feasible (scipy linprog).
"""
import math
import os

import numpy as np
import pytest
from scipy.optimize import linprog

from oracle import mjcf_ref
from oracle import oracle as O
from tests.conftest import SCENES

PLANE, SPHERE, CYL, BOX = 0, 2, 5, 6


def quat_axis(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    return [math.cos(ang / 2)] + list(math.sin(ang / 2) * axis)


def model_of(static, moving):
    """World with static geoms + one free body (qpos[0:7]) carrying `moving` geoms.

    Each geom: (type, size3, pos3, quat4[, margin]) in its body frame."""
    bodies = [(-1, -1, -1), (0, 0, 0)]
    geoms = [(0, g) for g in static] + [(1, g) for g in moving]
    m = dict(body_parent=[-1, 0], body_jnt_type=[-1, 0], body_qpos_adr=[-1, 0],
             body_pos=[[0, 0, 0], [0, 0, 0]], body_quat=[[1, 0, 0, 0], [1, 0, 0, 0]],
             geom_type=[g[0] for _, g in geoms], geom_body=[b for b, _ in geoms],
             geom_contype=[1] * len(geoms), geom_conaffinity=[1] * len(geoms),
             geom_size=[list(g[1]) + [0] * (3 - len(g[1])) for _, g in geoms],
             geom_pos=[g[2] for _, g in geoms], geom_quat=[g[3] for _, g in geoms],
             geom_margin=[g[4] if len(g) > 4 else 0.0 for _, g in geoms],
             exclude=np.zeros((0, 2), np.int32), qpos0=[0, 0, 0, 1, 0, 0, 0])
    del bodies
    return m


def contacts(static, moving, pos, quat=(1, 0, 0, 0), count_static=False):
    s = O.Scene(model_of(static, moving), 0, 7)
    return s.contacts(np.array(list(pos) + list(quat)), count_static)


FLOOR = (PLANE, (0, 0, 0.05), (0, 0, 0), (1, 0, 0, 0))


def test_box_on_plane_corner_contacts():
    box = (BOX, (0.1, 0.2, 0.3), (0, 0, 0), (1, 0, 0, 0))
    n, cost, nd = contacts([FLOOR], [box], (0, 0, 0.25))  # 4 bottom corners 0.05 deep
    assert (n, nd) == (4, 4)
    assert cost == pytest.approx(4 * -1.0 / (0.25 + 1e-4), rel=1e-15)
    assert contacts([FLOOR], [box], (0, 0, 0.2995))[:3:2] == (4, 0)  # shallow: contact, not deep
    # touching: MuJoCo's colliders drop a contact only when dist > margin (dist == 0 counts)
    assert contacts([FLOOR], [box], (0, 0, 0.3))[0] == 4
    assert contacts([FLOOR], [box], (0, 0, 0.3001))[0] == 0
    assert contacts([FLOOR], [box], (0, 0, 0.0))[0] == 4  # fully below: capped at 4 (MuJoCo)
    tilted = contacts([FLOOR], [box], (0, 0, 0.3), quat_axis([1, 0, 0], 0.1))
    assert tilted[0] == 2  # one edge dips below


def test_margin_activates_contact():
    box = (BOX, (0.1, 0.1, 0.1), (0, 0, 0), (1, 0, 0, 0), 0.01)
    assert contacts([FLOOR], [box], (0, 0, 0.105))[0] == 4   # 0.005 gap < margin 0.01
    assert contacts([FLOOR], [box], (0, 0, 0.115))[0] == 0


def test_sphere_and_cylinder_on_plane():
    sph = (SPHERE, (0.1,), (0, 0, 0), (1, 0, 0, 0))
    assert contacts([FLOOR], [sph], (0, 0, 0.05))[:3:2] == (1, 1)
    assert contacts([FLOOR], [sph], (0, 0, 0.11))[0] == 0
    cyl = (CYL, (0.05, 0.1), (0, 0, 0), (1, 0, 0, 0))
    # standing 1 cm deep: the lower cap's "deepest rim point" (any, the rim is level) and the two
    # triangle points of mjc_PlaneCylinder, all 1 cm deep
    assert contacts([FLOOR], [cyl], (0, 0, 0.09))[:3:2] == (3, 3)
    lying = quat_axis([1, 0, 0], math.pi / 2)
    # lying 1 cm deep: both caps' lowest rim points; the triangle points sit 2.5 cm above
    assert contacts([FLOOR], [cyl], (0, 0, 0.04), lying)[:3:2] == (2, 2)
    assert contacts([FLOOR], [cyl], (0, 0, 0.0495), lying)[:3:2] == (2, 0)  # 0.5 mm: 2 contacts, not deep


def mj_plane_box_count(h, R, e, margin):
    """Contacts of a box over the z = 0 plane by the rule of MuJoCo's published mjc_PlaneBox
    (centre height h, rotation R, half extents e): corners in bit order, skip when
    dist + ldist > margin or ldist > 0, at most 4; returns (count, deep count)."""
    n = d = 0
    for i in range(8):
        v = np.array([e[0] if i & 1 else -e[0], e[1] if i & 2 else -e[1], e[2] if i & 4 else -e[2]])
        ld = (R @ v)[2]
        if h + ld > margin or ld > 0:
            continue
        n += 1
        d += (h + ld) < -1e-3
        if n >= 4:
            break
    return n, d


def mj_plane_cyl_count(h, axis, r, hh, margin):
    """Contacts of a cylinder over the z = 0 plane by the rule of MuJoCo's published
    mjc_PlaneCylinder: the near cap's deepest rim point first (none at all when it is above the
    margin), the far cap's, and two triangle points on the near cap at -prjvec / 2."""
    nrm = np.array([0.0, 0.0, 1.0])
    axis = np.asarray(axis, float)
    pa = nrm @ axis
    if pa > 0:
        axis, pa = -axis, -pa
    vec = axis * pa - nrm
    ln = np.linalg.norm(vec)
    prjvec = (vec * (r / ln)) @ nrm if ln > 1e-15 else 0.0
    pa *= hh
    pts = [h + pa + prjvec, h - pa + prjvec, h + pa - 0.5 * prjvec, h + pa - 0.5 * prjvec]
    if pts[0] > margin:
        return 0, 0
    keep = [pts[0]] + ([pts[1]] if pts[1] <= margin else []) + (pts[2:] if pts[2] <= margin else [])
    return len(keep), sum(p < -1e-3 for p in keep)


def test_plane_box_and_cylinder_match_mujoco_rules():
    """Random boxes and cylinders around the floor: the oracle's contact and deep-contact counts
    equal the published MuJoCo plane colliders' rules restated independently above (counts,
    margin boundary, the corner half turned away from the plane, the cylinder triangle points)."""
    rng = np.random.default_rng(5)
    for trial in range(300):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        margin = [0.0, 0.002][trial % 2]
        e = rng.uniform(0.02, 0.2, size=3)
        h = rng.uniform(-0.3, 0.3)
        box = (BOX, tuple(e), (0, 0, 0), (1, 0, 0, 0), margin)
        got = contacts([FLOOR], [box], (0, 0, h), tuple(q))
        assert (got[0], got[2]) == mj_plane_box_count(h, R, e, margin), trial
        r, hh = rng.uniform(0.02, 0.1), rng.uniform(0.02, 0.2)
        cyl = (CYL, (r, hh), (0, 0, 0), (1, 0, 0, 0), margin)
        got = contacts([FLOOR], [cyl], (0, 0, h), tuple(q))
        assert (got[0], got[2]) == mj_plane_cyl_count(h, R[:, 2], r, hh, margin), trial


def test_box_box_axis_aligned():
    a = (BOX, (0.5, 0.5, 0.5), (0, 0, 0), (1, 0, 0, 0))
    # face against face, 0.1 deep: the clipped manifold has the 4 incident corners, all deep
    # (n counts the pair: SamplingPathPlanner feasibility only needs n > 0)
    assert contacts([a], [a], (0.9, 0, 0))[:3:2] == (1, 4)
    assert contacts([a], [a], (0.9995, 0, 0))[:3:2] == (1, 0)  # overlap 5e-4: not deep
    assert contacts([a], [a], (1.0, 0, 0))[0] == 0
    assert contacts([a], [a], (1.1, 0, 0))[0] == 0
    am = (BOX, (0.5, 0.5, 0.5), (0, 0, 0), (1, 0, 0, 0), 0.001)
    assert contacts([a], [am], (1.0005, 0, 0))[0] == 1
    # rotated 45 deg about z: reach along x is 0.5 * sqrt(2)
    r = quat_axis([0, 0, 1], math.pi / 4)
    assert contacts([a], [a], (0.5 + 0.5 * math.sqrt(2) - 1e-3, 0, 0), r)[0] == 1
    assert contacts([a], [a], (0.5 + 0.5 * math.sqrt(2) + 1e-3, 0, 0), r)[0] == 0


def _lp_intersect(pa, Ra, ea, pb, Rb, eb):
    A = np.vstack([Ra.T, -Ra.T, Rb.T, -Rb.T])
    b = np.concatenate([ea + Ra.T @ pa, ea - Ra.T @ pa, eb + Rb.T @ pb, eb - Rb.T @ pb])
    res = linprog(np.zeros(3), A_ub=A, b_ub=b, bounds=[(None, None)] * 3, method="highs")
    return res.status == 0


def _qmat(q):
    w, x, y, z = q
    return np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])


def test_box_box_sat_matches_lp_intersection():
    """Random oriented boxes: SAT contact (margin 0) == exact LP intersection (incl. edge-edge)."""
    rng = np.random.default_rng(42)
    agree, n = 0, 0
    for _ in range(400):
        ea, eb = rng.uniform(0.05, 0.3, 3), rng.uniform(0.05, 0.3, 3)
        qa, qb = rng.normal(size=4), rng.normal(size=4)
        qa, qb = qa / np.linalg.norm(qa), qb / np.linalg.norm(qb)
        pb = rng.uniform(-0.5, 0.5, 3)
        lp = _lp_intersect(np.zeros(3), _qmat(qa), ea, pb, _qmat(qb), eb)
        # skip near-touching cases where the LP's tolerance decides
        shrunk = _lp_intersect(np.zeros(3), _qmat(qa), ea * (1 - 1e-6), pb, _qmat(qb), eb * (1 - 1e-6))
        grown = _lp_intersect(np.zeros(3), _qmat(qa), ea * (1 + 1e-6), pb, _qmat(qb), eb * (1 + 1e-6))
        if shrunk != grown:
            continue
        sat = contacts([(BOX, ea, (0, 0, 0), qa)], [(BOX, eb, (0, 0, 0), (1, 0, 0, 0))], pb, qb)[0] > 0
        n += 1
        agree += sat == lp
    assert n > 350 and agree == n


def test_sphere_box_distance():
    box = (BOX, (0.2, 0.2, 0.2), (0, 0, 0), (1, 0, 0, 0))
    sph = (SPHERE, (0.1,), (0, 0, 0), (1, 0, 0, 0))
    assert contacts([box], [sph], (0.29, 0, 0))[0] == 1
    assert contacts([box], [sph], (0.31, 0, 0))[0] == 0
    d = 0.1 / math.sqrt(2)  # corner region: distance to edge (0.2, 0.2) along the diagonal
    assert contacts([box], [sph], (0.2 + d * 0.99, 0.2 + d * 0.99, 0))[0] == 1
    assert contacts([box], [sph], (0.2 + d * 1.01, 0.2 + d * 1.01, 0))[0] == 0


def test_cylinder_box_sat():
    box = (BOX, (0.2, 0.2, 0.05), (0, 0, 0), (1, 0, 0, 0))
    cyl = (CYL, (0.05, 0.1), (0, 0, 0), (1, 0, 0, 0))
    assert contacts([box], [cyl], (0, 0, 0.14))[:3:2] == (1, 1)      # standing on top, 10 mm deep
    assert contacts([box], [cyl], (0, 0, 0.151))[0] == 0
    assert contacts([box], [cyl], (0.24, 0, 0.0))[0] == 1           # beside, rim overlapping
    assert contacts([box], [cyl], (0.26, 0, 0.0))[0] == 0


def test_broadphase_sphere_semantics():
    """Pairs whose bounding spheres (+margin) are apart are skipped (MuJoCo rbound test)."""
    a = (BOX, (0.1, 0.1, 0.1), (0, 0, 0), (1, 0, 0, 0), 0.5)
    # SAT separation along x is 0.45 < margin 0.5, but centres are 0.65 > 2*0.1732+0.5 apart?
    # |c| = 0.65*sqrt(3) = 1.1258 > 0.3464 + 0.5 -> culled, no contact
    assert contacts([a], [a], (0.65, 0.65, 0.65))[0] == 0
    assert contacts([a], [a], (0.6, 0, 0))[0] == 1


@pytest.fixture(scope="module")
def robocrane():
    return mjcf_ref.load(os.path.join(SCENES, "robocrane.xml"))


def test_robocrane_pair_filter(robocrane):
    s = O.Scene(robocrane, 0, 7)
    n_mov, n_stat = s.npairs()
    # block_green vs floor, table, cyan, magenta + 6 gripper primitives (contype 1)
    assert n_mov == 10
    assert n_stat > 0
    names = robocrane["geom_names"]
    q = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    xp, xm = s.fk(q)
    g = names.index("block_green/block_green_geom")
    np.testing.assert_allclose(xp[g], [0.5, 0.15, 0.156], atol=1e-15)
    np.testing.assert_allclose(xm[g].reshape(3, 3), [[0, -1, 0], [1, 0, 0], [0, 0, 1]], atol=1e-15)
    t = names.index("wall/table_geom")
    np.testing.assert_allclose(xp[t], [0.5, 0, 0.058], atol=1e-15)
    # start/end hover 20 mm over the table, the straight line crosses the brick stack
    assert s.contacts(q)[0] == 0
    assert s.contacts(np.array([0.5, 0.05, 0.136, 0.707, 0, 0, 0.707]))[0] >= 1
    assert s.contacts(np.array([0.5, 0.05, 0.25, 0.707, 0, 0, 0.707]))[0] == 0
    # resting bodies (blue/orange on the table, stacked bricks) touch at dist 0: no contact
    assert s.contacts(q, count_static=True)[0] == 0


def test_stacking_tsp_cost(robocrane):
    m = mjcf_ref.load(os.path.join(SCENES, "stacking.xml"))
    s = O.Scene(m, 1, 1)  # block1
    assert s.npairs() == (3, 3)  # block1 vs floor/block2/block3; block2-floor, block3-floor, 2-3
    n, cost, nd = s.contacts(np.array([0.205, 0.0, 0.12, 0.0]))
    # block1 clear of everything; block2 and block3 rest on the floor at distance exactly 0,
    # which MuJoCo's plane-box collider counts (4 corners each, none deep): no cost
    assert (n, cost, nd) == (8, 0.0, 0)
    # overlapping block2 by 50 mm in x, face to face: the manifold's 4 corners are all deep
    # (Collision.h:89-101 adds one term per contact), centre distance 0.15
    n, cost, nd = s.contacts(np.array([0.15, 0.0, 0.1, 0.0]))
    assert nd == 4 and cost == pytest.approx(4 * -1.0 / (0.15 + 1e-4), rel=1e-14)

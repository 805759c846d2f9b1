"""ctypes wrapper around oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
The product (sspp_amd/, sspp/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liboracle.so")

_d = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u8 = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i32 = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


class _Model(C.Structure):
    _fields_ = [
        ("nbody", C.c_int), ("body_parent", C.c_void_p), ("body_jnt_type", C.c_void_p),
        ("body_qpos_adr", C.c_void_p), ("body_pos", C.c_void_p), ("body_quat", C.c_void_p),
        ("ngeom", C.c_int), ("geom_type", C.c_void_p), ("geom_body", C.c_void_p),
        ("geom_contype", C.c_void_p), ("geom_conaffinity", C.c_void_p),
        ("geom_size", C.c_void_p), ("geom_pos", C.c_void_p), ("geom_quat", C.c_void_p),
        ("geom_margin", C.c_void_p), ("nexclude", C.c_int), ("exclude", C.c_void_p),
        ("nq", C.c_int), ("qpos0", C.c_void_p),
    ]


class _CesCfg(C.Structure):
    _fields_ = [("K", C.c_int), ("frac", C.c_double), ("inc", C.c_double), ("dec", C.c_double),
                ("sigma_floor", C.c_double), ("var_beta", C.c_double), ("mean_lr", C.c_double),
                ("sd_min", C.c_double), ("sd_max", C.c_double), ("dist_z_min", C.c_double),
                ("lo", C.c_double * 4), ("hi", C.c_double * 4), ("sequential", C.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        L.or_scene_create.restype = C.c_void_p
        L.or_scene_create.argtypes = [C.POINTER(_Model), C.c_int, C.c_int]
        L.or_scene_destroy.argtypes = [C.c_void_p]
        L.or_scene_npairs.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.or_knot_averaging.argtypes = [_d, C.c_int, C.c_int, _d]
        L.or_span.argtypes = [C.c_double, C.c_int, _d, C.c_int]
        L.or_basis.argtypes = [C.c_double, C.c_int, _d, C.c_int, _d]
        L.or_spline_eval.argtypes = [_d, C.c_int, C.c_int, _d, C.c_int, C.c_double, _d]
        L.or_interpolate.argtypes = [_d, C.c_int, C.c_int, C.c_int, _d, _d, _d]
        L.or_py_knot_vector.argtypes = [C.c_int, C.c_int, _d]
        L.or_py_B.restype = C.c_double
        L.or_py_B.argtypes = [C.c_double, C.c_int, C.c_int, _d]
        L.or_py_bspline.argtypes = [C.c_double, _d, C.c_int, _d, C.c_int, C.c_int, _d]
        L.or_normal_pair.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                     C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.or_normal_pair_libm.argtypes = L.or_normal_pair.argtypes
        L.or_normal_quad.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, _d]
        L.or_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint32)]
        L.or_sample_sspp.argtypes = [_d, C.c_int, C.c_int, C.c_int, C.c_double, _d, C.c_uint64,
                                     C.c_int64, C.c_int64, _d, C.c_int]
        L.or_sample_tsp.argtypes = [_d, _d, C.c_int, _d, _d, C.c_double, C.c_uint64, C.c_int64,
                                    C.c_int64, _d]
        L.or_point_contacts.argtypes = [C.c_void_p, _d, C.c_int, C.POINTER(C.c_double),
                                        C.POINTER(C.c_int)]
        L.or_fk_geoms.argtypes = [C.c_void_p, _d, _d, _d]
        L.or_canon_sum.restype = C.c_double
        L.or_canon_sum.argtypes = [_d, C.c_int, C.c_int]
        L.or_lanes_for.argtypes = [C.c_int]
        L.or_sspp_score.argtypes = [C.c_void_p, _d, C.c_int, C.c_int, _d, C.c_int, C.c_int,
                                    C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    _d, _u8]
        L.or_argmin.restype = C.c_int64
        L.or_argmin.argtypes = [_d, _u8, C.c_int64, C.POINTER(C.c_double)]
        L.or_tsp_score.argtypes = [C.c_void_p, _d, _d, _d, C.c_int, C.c_int64, C.c_int,
                                   C.c_double, C.c_int, C.c_int, _d, _d, _d, _u8, _d]
        L.or_ces_update.restype = C.c_int
        L.or_ces_update.argtypes = [C.POINTER(_CesCfg), _d, _u8, _d, C.c_int64, _d, _d, _d,
                                    C.POINTER(C.c_int), _i32, C.POINTER(C.c_int),
                                    C.POINTER(C.c_int64)]
        L.or_tsp_best.restype = C.c_int64
        L.or_tsp_best.argtypes = [_d, _u8, C.c_int64, C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _f64(x, shape=None):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    return a.reshape(shape) if shape is not None else a


# ------------------------------------------------------------------ splines
def knot_averaging(u, p):
    u = _f64(u)
    k = np.zeros(len(u) + p + 1)
    lib().or_knot_averaging(u, len(u), p, k)
    return k


def span(u, p, knots):
    knots = _f64(knots)
    return lib().or_span(float(u), p, knots, len(knots))


def basis(u, p, knots):
    knots = _f64(knots)
    N = np.zeros(p + 1)
    lib().or_basis(float(u), p, knots, len(knots), N)
    return N


def spline_eval(knots, p, ctrl, u):
    knots, ctrl = _f64(knots), _f64(ctrl)
    out = np.zeros(ctrl.shape[1])
    lib().or_spline_eval(knots, len(knots), p, ctrl, ctrl.shape[1], float(u), out)
    return out


def interpolate(pts, p, u):
    pts, u = _f64(pts), _f64(u)
    n, D = pts.shape
    knots = np.zeros(n + p + 1)
    ctrl = np.zeros((n, D))
    rc = lib().or_interpolate(pts, n, D, p, u, knots, ctrl)
    if rc != 0:
        raise RuntimeError("or_interpolate failed %d" % rc)
    return knots, ctrl


def py_knot_vector(n, k):
    t = np.zeros(n + k + 1)
    lib().or_py_knot_vector(n, k, t)
    return t


def py_bspline(theta, t, c, k):
    t, c = _f64(t), _f64(c)
    if c.ndim == 1:
        c = c.reshape(-1, 1)
    out = np.zeros(c.shape[1])
    lib().or_py_bspline(float(theta), t, len(t), c, c.shape[1], k, out)
    return out


# ------------------------------------------------------------------ RNG / sampling
def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return list(o)


def normal_quad(seed, cand, idx, stream):
    """The SamplingPathPlanner sampler's four FP32 Box-Muller normals of one Philox call."""
    z = np.zeros(4)
    lib().or_normal_quad(seed, cand, idx, stream, z)
    return z


def normal_pair(seed, cand, idx, stream, libm=False):
    """Two FP64 Box-Muller normals of one Philox call (the kernels' normal_pair); libm=True:
    the same transform through libm log / sin / cos (accuracy reference)."""
    z0, z1 = C.c_double(), C.c_double()
    f = lib().or_normal_pair_libm if libm else lib().or_normal_pair
    f(seed, cand, idx, stream, C.byref(z0), C.byref(z1))
    return z0.value, z1.value


SAMPLER_FP64, SAMPLER_FP32 = 0, 1


def sample_sspp(init_ctrl, p, sigma, limits, seed, first, B, sampler=SAMPLER_FP64):
    """sampleWithNoise (include/sspp.h:114-130) for candidate ids [first, first + B);
    sampler 0: FP64 Box-Muller pairs (default), 1: the opt-in FP32 quads."""
    init_ctrl = _f64(init_ctrl)
    n, D = init_ctrl.shape
    out = np.zeros((B, n, D))
    lib().or_sample_sspp(init_ctrl, n, D, p, float(sigma), _f64(limits).reshape(D), seed,
                         first, B, out, int(sampler))
    return out


def sample_tsp(mean, sigma, lo, hi, z_min, seed, first, B):
    mean, sigma = _f64(mean).reshape(-1, 4), _f64(sigma).reshape(-1, 4)
    K = mean.shape[0]
    out = np.zeros((B, K, 4))
    lib().or_sample_tsp(mean, sigma, K, _f64(lo).reshape(4), _f64(hi).reshape(4),
                        float(z_min), seed, first, B, out)
    return out


# ------------------------------------------------------------------ scene
class Scene:
    """Oracle scene: model + moving set. mode 0 = qpos window of `arg` dofs, mode 1 = body id."""

    def __init__(self, model, mode, arg, skip_types=()):
        """skip_types: geom types made non-collidable (contype = conaffinity = 0), for tests
        that show which candidates a pair type decides."""
        self._keep = {}
        m = _Model()
        if skip_types:
            model = dict(model)
            off = np.isin(np.asarray(model["geom_type"]), list(skip_types))
            model["geom_contype"] = np.where(off, 0, model["geom_contype"])
            model["geom_conaffinity"] = np.where(off, 0, model["geom_conaffinity"])

        def put(name, arr, dtype):
            a = np.ascontiguousarray(np.asarray(arr, dtype=dtype))
            self._keep[name] = a
            return a.ctypes.data_as(C.c_void_p)

        m.nbody = len(model["body_parent"])
        m.body_parent = put("bp", model["body_parent"], np.int32)
        m.body_jnt_type = put("bj", model["body_jnt_type"], np.int32)
        m.body_qpos_adr = put("ba", model["body_qpos_adr"], np.int32)
        m.body_pos = put("bpos", model["body_pos"], np.float64)
        m.body_quat = put("bq", model["body_quat"], np.float64)
        m.ngeom = len(model["geom_type"])
        m.geom_type = put("gt", model["geom_type"], np.int32)
        m.geom_body = put("gb", model["geom_body"], np.int32)
        m.geom_contype = put("gc", model["geom_contype"], np.int32)
        m.geom_conaffinity = put("ga", model["geom_conaffinity"], np.int32)
        m.geom_size = put("gs", model["geom_size"], np.float64)
        m.geom_pos = put("gp", model["geom_pos"], np.float64)
        m.geom_quat = put("gq", model["geom_quat"], np.float64)
        m.geom_margin = put("gm", model["geom_margin"], np.float64)
        ex = np.asarray(model["exclude"], np.int32).reshape(-1, 2)
        m.nexclude = ex.shape[0]
        m.exclude = put("ex", ex, np.int32)
        m.nq = len(model["qpos0"])
        m.qpos0 = put("q0", model["qpos0"] if len(model["qpos0"]) else [0.0], np.float64)
        self._m = m
        self.mode, self.arg = mode, arg
        self.ngeom = m.ngeom
        self.ptr = lib().or_scene_create(C.byref(m), mode, arg)
        if not self.ptr:
            raise RuntimeError("or_scene_create failed")

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.or_scene_destroy(self.ptr)
            self.ptr = None

    def npairs(self):
        a, b = C.c_int(), C.c_int()
        lib().or_scene_npairs(self.ptr, C.byref(a), C.byref(b))
        return a.value, b.value

    def contacts(self, q, count_static=False):
        c, nd = C.c_double(), C.c_int()
        n = lib().or_point_contacts(self.ptr, _f64(q), int(count_static), C.byref(c), C.byref(nd))
        return n, c.value, nd.value

    def fk(self, q):
        xp = np.zeros((self.ngeom, 3))
        xm = np.zeros((self.ngeom, 9))
        lib().or_fk_geoms(self.ptr, _f64(q), xp, xm)
        return xp, xm


# ------------------------------------------------------------------ scoring
def canon_sum(x, lanes=None):
    x = _f64(x)
    if lanes is None:
        lanes = lib().or_lanes_for(len(x))
    return lib().or_canon_sum(x, len(x), lanes)


def sspp_score(scene, knots, p, ctrl, W, count_static=False, sequential=False, nthreads=0,
               arc_all=False):
    """checkCollision + computeArcLength per candidate.  arc_all=False follows findBestPath
    (include/sspp.h:171-192): only collision-free candidates get an arc length, the rest +inf."""
    knots, ctrl = _f64(knots), _f64(ctrl)
    B, n, D = ctrl.shape
    arc = np.zeros(B)
    feas = np.zeros(B, np.uint8)
    rc = lib().or_sspp_score(scene.ptr if scene is not None else None, knots, len(knots), p,
                             ctrl, n, D, B, W, int(count_static), int(sequential), nthreads,
                             int(bool(arc_all)), arc, feas)
    if rc != 0:
        raise RuntimeError("or_sspp_score failed %d" % rc)
    return arc, feas


def argmin(cost, feasible):
    cost = _f64(cost)
    f = np.ascontiguousarray(np.asarray(feasible, np.uint8))
    best = C.c_double()
    idx = lib().or_argmin(cost, f, len(cost), C.byref(best))
    return int(idx), best.value


def tsp_score(scene, start, end, vias, cp, w_collision=1.0, sequential=False, nthreads=0):
    vias = _f64(vias)
    B, K, _ = vias.shape
    L, Cnf, Cwf, cost = (np.zeros(B) for _ in range(4))
    st = np.zeros(B, np.uint8)
    rc = lib().or_tsp_score(scene.ptr, _f64(start).reshape(4), _f64(end).reshape(4), vias, K, B,
                            cp, float(w_collision), int(sequential), nthreads, L, Cnf, Cwf, st,
                            cost)
    if rc != 0:
        raise RuntimeError("or_tsp_score failed %d" % rc)
    return L, Cnf, Cwf, st, cost


def tsp_best(cost, status):
    cost = _f64(cost)
    st = np.ascontiguousarray(np.asarray(status, np.uint8))
    best = C.c_double()
    idx = lib().or_tsp_best(cost, st, len(cost), C.byref(best))
    return int(idx), best.value


# ------------------------------------------------------------------ TaskSpacePlanner CES
CES_DEFAULTS = dict(frac=0.3, inc=1.5, dec=0.95, sigma_floor=0.0, var_beta=0.2, mean_lr=0.5,
                    sd_min=0.01, sd_max=0.5, dist_z_min=0.3, lo=(-2.0,) * 4, hi=(2.0,) * 4)


def ces_update(cost, status, vias, mean, sigma, last_best, has_best, sequential=False, **cfg):
    """tsp::Planner::plan's update (tsp_planner.h:121-142) on one iteration's candidate list.
    Returns (mean, sigma, last_best, has_best, n_success, elites, best_slot)."""
    c = dict(CES_DEFAULTS, **cfg)
    vias = _f64(vias)
    n, K = vias.shape[0], vias.shape[1]
    cc = _CesCfg(K=K, frac=c["frac"], inc=c["inc"], dec=c["dec"], sigma_floor=c["sigma_floor"],
                 var_beta=c["var_beta"], mean_lr=c["mean_lr"], sd_min=c["sd_min"],
                 sd_max=c["sd_max"], dist_z_min=c["dist_z_min"],
                 lo=(C.c_double * 4)(*c["lo"]), hi=(C.c_double * 4)(*c["hi"]),
                 sequential=int(bool(sequential)))
    mean, sigma = _f64(mean).reshape(K, 4).copy(), _f64(sigma).reshape(K, 4).copy()
    lb = _f64(last_best).reshape(K, 4).copy()
    hb = C.c_int(int(bool(has_best)))
    elites = np.zeros(max(n, 1), np.int32)
    ne, bs = C.c_int(), C.c_int64()
    ns = lib().or_ces_update(C.byref(cc), _f64(cost), np.ascontiguousarray(status, np.uint8), vias,
                             n, mean, sigma, lb, C.byref(hb), elites, C.byref(ne), C.byref(bs))
    return mean, sigma, lb, bool(hb.value), ns, elites[:ne.value].copy(), int(bs.value)


def ces_reset(start, end, total_points, z_min=0.0, dist_z_min=0.3, sigma0=0.3, sd_min=0.01,
              sd_max=0.5, sigma_floor=0.0, lo=(-2.0,) * 4, hi=(2.0,) * 4):
    """Planner::reset + Distribution::reset (tsp_planner.h:54-69, tsp_distribution.h:16-29)."""
    K = total_points - 2
    start, end = _f64(start), _f64(end)
    mean = np.zeros((K, 4))
    for i in range(K):
        t = (i + 1) / (total_points - 1)
        for d in range(4):
            v = (1.0 - t) * start[d] + t * end[d]
            if d == 2:
                v = max(v, z_min)
                v = v if v >= dist_z_min else dist_z_min
            v = lo[d] if v < lo[d] else (hi[d] if hi[d] < v else v)
            mean[i, d] = v
    s = sigma0
    s = sd_min if s < sd_min else s
    s = sd_max if s > sd_max else s
    s = sigma_floor if s < sigma_floor else s
    return mean, np.full((K, 4), s)


def ces_plan(scene, start, end, iterations, samples, checks, total_points=3, seed=0x5EED,
             z_min=0.0, w_collision=1.0, nthreads=0, sequential=False, **cfg):
    """CPU restatement of TaskSpacePlanner::plan(start, end, iterate) repeated `iterations`
    times (first call iterate=False): seeds, evaluation, update.  Same Philox ids as the GPU
    (iteration t samples t * samples + [0, samples)).  Returns the per-iteration records."""
    c = dict(CES_DEFAULTS, **cfg)
    K = total_points - 2
    mean, sigma = ces_reset(start, end, total_points, z_min, c["dist_z_min"], 0.3, c["sd_min"],
                            c["sd_max"], c["sigma_floor"], c["lo"], c["hi"])
    lb, hb = np.zeros((K, 4)), False
    out = []
    for t in range(iterations):
        seeds = [np.where(np.arange(4) == 2, np.maximum(mean, z_min), mean)]
        if hb:
            seeds.append(lb.copy())
        smp = sample_tsp(mean, sigma, c["lo"], c["hi"], z_min, seed, t * samples, samples)
        vias = np.concatenate([np.array(seeds).reshape(-1, K, 4), smp.reshape(-1, K, 4)])
        L, Cnf, Cwf, st, cost = tsp_score(scene, start, end, vias, checks, w_collision,
                                          nthreads=nthreads)
        rec = dict(vias=vias, L=L, C_nf=Cnf, C_wf=Cwf, status=st, cost=cost,
                   mean_in=mean.copy(), sigma_in=sigma.copy())
        mean, sigma, lb, hb, ns, el, bs = ces_update(cost, st, vias, mean, sigma, lb, hb,
                                                     sequential=sequential, **cfg)
        rec.update(mean=mean, sigma=sigma, last_best=lb, has_best=hb, n_success=ns, elites=el,
                   best_slot=bs)
        out.append(rec)
    return out

"""Python host objects over the C ABI: Model, Scene, SsppJob, TspJob.

Device buffers are torch CUDA tensors (torch is plumbing here: HBM allocation, streams and
torch.distributed); every computation runs in the HIP kernels of libsspp_hip.so.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import (Best, CesBuffers, CesConfig, CesInfo, CesState, ModelView, SceneInfo,
                   SsppArgs, TspArgs, check, lib)

DEFAULT_SEED = 0x5EED
SAMPLER_FP64, SAMPLER_FP32 = 0, 1  # sspp_sspp_args::sampler


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(x, n=None):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if n is not None and a.size != n:
        raise ValueError("expected %d values, got %d" % (n, a.size))
    return a


def _torch():
    import torch  # noqa: WPS433 (plumbing only)
    return torch


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(stream):
    if stream is None:
        torch = _torch()
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def best_tensor(device="cuda"):
    """A device buffer for one sspp_best record (4 x int64; cost is the bits of field 0)."""
    return _torch().zeros(4, dtype=_torch().int64, device=device)


def check_records(t):
    """Refuse result records that report lost work: any record (int64 [..., 4] tensor or array)
    whose `reserved` field is non-zero raises SsppError through sspp_best_check
    (SSPP_E_INCOMPLETE).  Returns the records as a numpy int64 [n, 4] array."""
    a = t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)
    a = np.ascontiguousarray(a.astype(np.int64).reshape(-1, 4))
    if a.shape[0] and np.any(a[:, 3] != 0):
        check(lib().sspp_best_check(a.ctypes.data_as(C.POINTER(Best)), int(a.shape[0])), "result record")
    return a


def decode_best(t):
    """(cost, index, count) from a best buffer (torch tensor or numpy int64[4]); a record that
    reports lost work raises SsppError (check_records)."""
    a = check_records(t)[0]
    cost = a[:1].view(np.float64)[0]
    return float(cost), int(a[1]), int(a[2])


def reduce_best(parts):
    """Global argmin over gathered per-rank records (cost, index, count[, reserved]): lowest
    cost, lowest id on ties; a record with reserved != 0 raises SsppError."""
    arr = (Best * len(parts))()
    for i, p in enumerate(parts):
        arr[i].cost, arr[i].index, arr[i].count = p[0], p[1], p[2]
        arr[i].reserved = p[3] if len(p) > 3 else 0
    out = Best()
    check(lib().sspp_best_reduce(arr, len(parts), C.byref(out)), "sspp_best_reduce")
    return out.cost, out.index, out.count


def reduce_best_device(parts, out, stream=None):
    """Device argmin over gathered records: parts int64 [n, 4] tensor -> out int64 [4]."""
    n = parts.shape[0]
    check(lib().sspp_best_reduce_device(_ptr(parts), int(n), _ptr(out), _stream(stream)),
          "sspp_best_reduce_device")


class Model:
    """Parsed MJCF scene (SamplingPathPlanner(xml_path) semantics: the string is a path)."""

    def __init__(self, xml_path):
        h = C.c_void_p()
        check(lib().sspp_model_load_mjcf(str(xml_path).encode(), C.byref(h)), "load MJCF")
        self._h = h
        self.path = str(xml_path)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.sspp_model_free(self._h)
            self._h = None

    def arrays(self):
        v = ModelView()
        check(lib().sspp_model_view_get(self._h, C.byref(v)), "model view")

        def arr(p, n, dt, shape):
            if n == 0:
                return np.zeros(shape, dt)
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt).reshape(shape)

        nb, ng, ne, nq = v.nbody, v.ngeom, v.nexclude, v.nq
        return dict(
            body_parent=arr(v.body_parent, nb, np.int32, (nb,)),
            body_jnt_type=arr(v.body_jnt_type, nb, np.int32, (nb,)),
            body_qpos_adr=arr(v.body_qpos_adr, nb, np.int32, (nb,)),
            body_pos=arr(v.body_pos, 3 * nb, np.float64, (nb, 3)),
            body_quat=arr(v.body_quat, 4 * nb, np.float64, (nb, 4)),
            geom_type=arr(v.geom_type, ng, np.int32, (ng,)),
            geom_body=arr(v.geom_body, ng, np.int32, (ng,)),
            geom_contype=arr(v.geom_contype, ng, np.int32, (ng,)),
            geom_conaffinity=arr(v.geom_conaffinity, ng, np.int32, (ng,)),
            geom_size=arr(v.geom_size, 3 * ng, np.float64, (ng, 3)),
            geom_pos=arr(v.geom_pos, 3 * ng, np.float64, (ng, 3)),
            geom_quat=arr(v.geom_quat, 4 * ng, np.float64, (ng, 4)),
            geom_margin=arr(v.geom_margin, ng, np.float64, (ng,)),
            exclude=arr(v.exclude, 2 * ne, np.int32, (ne, 2)),
            qpos0=arr(v.qpos0, nq, np.float64, (nq,)),
        )

    def body_id(self, name):
        return check(lib().sspp_model_body_id(self._h, name.encode()), "body lookup")

    def geom_id(self, name):
        return check(lib().sspp_model_geom_id(self._h, name.encode()), "geom lookup")

    def body_point(self, name):
        out = np.zeros(4)
        check(lib().sspp_model_body_point(self._h, name.encode(), _dptr(out)), "body point")
        return out


class Scene:
    """Model bound to its moving set, with device-resident geom/pair tables.  count_static: the
    SamplingPathPlanner feasibility counts the scene's static-static contacts too (the
    reference's whole-scene ncon, include/sspp.h:143-144; Q7); False ignores them.  The
    TaskSpacePlanner cost always includes them (Collision.h:89-101)."""

    def __init__(self, model, mode, arg, count_static=True):
        if isinstance(arg, str):
            arg = model.body_id(arg)
        h = C.c_void_p()
        check(lib().sspp_scene_create(model.handle, int(mode), int(arg), int(bool(count_static)),
                                      C.byref(h)), "scene create")
        self._h = h
        self.model = model  # keep alive
        self.mode, self.arg = mode, arg

    @property
    def handle(self):
        return self._h

    def info(self):
        i = SceneInfo()
        check(lib().sspp_scene_get_info(self._h, C.byref(i)), "scene info")
        return {k: getattr(i, k) for k, _ in SceneInfo._fields_}

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.sspp_scene_free(self._h)
            self._h = None


def interpolate(pts, degree, u):
    """Eigen SplineFitting::Interpolate (include/sspp.h:95): returns (knots, ctrl [n][D])."""
    pts = np.ascontiguousarray(np.asarray(pts, dtype=np.float64))
    n, D = pts.shape
    u = _f64(u, n)
    knots = np.zeros(n + degree + 1)
    ctrl = np.zeros((n, D))
    check(lib().sspp_interpolate(_dptr(pts), n, D, int(degree), _dptr(u), _dptr(knots),
                                 _dptr(ctrl)), "interpolate")
    return knots, ctrl


def spline_eval(knots, degree, ctrl, u):
    knots = _f64(knots)
    ctrl = np.ascontiguousarray(np.asarray(ctrl, dtype=np.float64))
    D = ctrl.shape[1]
    out = np.zeros(D)
    check(lib().sspp_spline_eval(_dptr(knots), knots.size, int(degree), _dptr(ctrl), D,
                                 float(u), _dptr(out)), "spline eval")
    return out


class _Job:
    _h = None

    def info(self):
        a, b, c, d = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
        check(lib().sspp_job_info(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)), "job info")
        return dict(lanes_per_candidate=a.value, candidates_per_block=b.value,
                    block_threads=c.value, lds_bytes=d.value)

    def set_option(self, key, value):
        """Explicit launch option (include/sspp_hip.h SSPP_OPT_*; tests and tuning)."""
        check(lib().sspp_job_set_option(self._h, int(key), int(value)), "job set_option")

    def get_option(self, key):
        v = C.c_int64()
        check(lib().sspp_job_get_option(self._h, int(key), C.byref(v)), "job get_option")
        return int(v.value)

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.sspp_job_free(self._h)
            self._h = None


class SsppJob(_Job):
    """SamplingPathPlanner::plan's candidate loop on the GPU (include/sspp.h:194-225)."""

    def __init__(self, scene, knots, degree, init_ctrl, sigma, limits, check_points,
                 seed=DEFAULT_SEED, max_batch=4096, arc_all=False, sampler=SAMPLER_FP64):
        """arc_all=False follows the reference: arc length only for collision-free candidates
        (findBestPath scores only successful paths), +inf for the others.  sampler: FP64
        Box-Muller normals (default, as std::normal_distribution<double>) or the opt-in FP32
        quads (SAMPLER_FP32)."""
        init_ctrl = np.ascontiguousarray(np.asarray(init_ctrl, dtype=np.float64))
        n, D = init_ctrl.shape
        self.knots = _f64(knots, n + degree + 1)
        self.init_ctrl = init_ctrl
        self.limits = _f64(limits, D)
        self.n, self.D, self.degree, self.W = n, D, int(degree), int(check_points)
        self.max_batch = int(max_batch)
        a = SsppArgs(knots=_dptr(self.knots), degree=self.degree, init_ctrl=_dptr(init_ctrl),
                     n_ctrl=n, dof=D, sigma=float(sigma), limits=_dptr(self.limits),
                     check_points=self.W, seed=int(seed) & (2 ** 64 - 1), arc_all=int(bool(arc_all)),
                     sampler=int(sampler))
        self.sampler = int(sampler)
        h = C.c_void_p()
        check(lib().sspp_job_create_sspp(scene.handle if scene is not None else None, C.byref(a),
                                         self.max_batch, C.byref(h)), "job create (sspp)")
        self._h = h
        self.scene = scene

    def alloc(self, B, device="cuda", with_ctrl=False):
        torch = _torch()
        out = dict(arc=torch.empty(B, dtype=torch.float64, device=device),
                   feasible=torch.empty(B, dtype=torch.uint8, device=device),
                   best=best_tensor(device))
        if with_ctrl:
            out["ctrl"] = torch.empty((B, self.n, self.D), dtype=torch.float64, device=device)
        return out

    def sample_score(self, first_id, B, arc, feasible, best, ctrl_out=None, stream=None):
        check(lib().sspp_job_sample_score(self._h, int(first_id), int(B), _ptr(arc), _ptr(feasible),
                                          _ptr(ctrl_out), _ptr(best), _stream(stream)),
              "sample_score")

    def score_ctrl(self, ctrl, first_id, arc, feasible, best, stream=None):
        B = ctrl.shape[0]
        check(lib().sspp_job_score_ctrl(self._h, _ptr(ctrl), int(first_id), int(B), _ptr(arc),
                                        _ptr(feasible), _ptr(best), _stream(stream)), "score_ctrl")

    def set_shape(self, nt=0, g1=0):
        """Force the k_sspp_c2f launch shape (threads per workgroup 64 / 256, phase-1 lanes per
        candidate); 0, 0 = chosen per launch.  Every shape gives the same results."""
        self.set_option(_lib.OPT_SHAPE_NT, nt)
        self.set_option(_lib.OPT_SHAPE_G1, g1)

    def config(self):
        """The job's effective configuration, read back from the library."""
        g = self.get_option
        return dict(sampler="fp32" if g(_lib.OPT_SAMPLER) else "fp64",
                    shape="%dx%d" % (g(_lib.OPT_LAST_NT), g(_lib.OPT_LAST_G1)),
                    pair_order={0: "scene", 1: "gap", 2: "hit"}[g(_lib.OPT_ORDER)],
                    waypoint_order={0: "bisection", 2: "hit"}[g(_lib.OPT_WP_ORDER)],
                    prepass_ms=g(_lib.OPT_PREPASS_US) / 1e3, sampled_pairs=g(_lib.OPT_NPAIRS),
                    cylinder_box=bool(g(_lib.OPT_CYLBOX)),
                    scan="fp32-filtered" if g(_lib.OPT_LAST_F32) else "fp64",
                    split=bool(g(_lib.OPT_LAST_SPLIT)))


class TspJob(_Job):
    """tsp::Planner::plan's evaluation loop on the GPU (include/sspp/tsp_planner.h:89-138)."""

    def __init__(self, scene, start, end, n_vias, check_points, mean=None, sigma=None,
                 lo=(-2, -2, -2, -2), hi=(2, 2, 2, 2), z_min=0.0, w_collision=1.0,
                 seed=DEFAULT_SEED, max_batch=4096, floor=(0.0, 0.01, 10.0)):
        K = int(n_vias)
        self.start, self.end = _f64(start, 4), _f64(end, 4)
        self.mean = _f64(mean if mean is not None else np.zeros((max(K, 1), 4)))
        self.sigma = _f64(sigma if sigma is not None else np.zeros((max(K, 1), 4)))
        self.lo, self.hi = _f64(lo, 4), _f64(hi, 4)
        self.K, self.cp, self.max_batch = K, int(check_points), int(max_batch)
        a = TspArgs(start=_dptr(self.start), end=_dptr(self.end), n_vias=K, check_points=self.cp,
                    w_collision=float(w_collision), mean=_dptr(self.mean), sigma=_dptr(self.sigma),
                    lo=_dptr(self.lo), hi=_dptr(self.hi), z_min=float(z_min),
                    seed=int(seed) & (2 ** 64 - 1), floor_z_min=float(floor[0]),
                    floor_margin=float(floor[1]), floor_scale=float(floor[2]))
        h = C.c_void_p()
        check(lib().sspp_job_create_tsp(scene.handle, C.byref(a), self.max_batch, C.byref(h)),
              "job create (tsp)")
        self._h = h
        self.scene = scene

    def alloc(self, B, device="cuda", with_vias=False):
        torch = _torch()
        f = lambda: torch.empty(B, dtype=torch.float64, device=device)  # noqa: E731
        out = dict(L=f(), Cnf=f(), Cwf=f(), cost=f(),
                   status=torch.empty(B, dtype=torch.uint8, device=device),
                   best=best_tensor(device))
        if with_vias:
            out["vias"] = torch.empty((B, max(self.K, 1), 4), dtype=torch.float64, device=device)
        return out

    def sample_score(self, first_id, B, L, Cnf, Cwf, status, cost, best, vias_out=None, stream=None):
        check(lib().sspp_job_tsp_sample_score(self._h, int(first_id), int(B), _ptr(L), _ptr(Cnf),
                                              _ptr(Cwf), _ptr(status), _ptr(cost), _ptr(vias_out),
                                              _ptr(best), _stream(stream)), "tsp sample_score")

    def score_vias(self, vias, first_id, L, Cnf, Cwf, status, cost, best, stream=None):
        B = vias.shape[0]
        check(lib().sspp_job_tsp_score_vias(self._h, _ptr(vias), int(first_id), int(B), _ptr(L),
                                            _ptr(Cnf), _ptr(Cwf), _ptr(status), _ptr(cost),
                                            _ptr(best), _stream(stream)), "tsp score_vias")


class SsppSteps:
    """Back-to-back SamplingPathPlanner steps enqueued by the C++ step executor
    (sspp_steps_enqueue_sspp): step i scores ids first_id + i * step_stride + [0, B); steps go
    steps_per_launch to a kernel launch, launch l to branch l % len(jobs) — jobs[b] with
    streams[b] and its scratch arc/feasible buffers (steps_per_launch * B entries each)."""

    def __init__(self, jobs, streams, B, arc_bufs, feas_bufs, steps_per_launch=1):
        nb = len(jobs)
        self._keep = (jobs, streams, arc_bufs, feas_bufs)
        self.arc_bufs, self.feas_bufs = arc_bufs, feas_bufs  # each branch's last launch's outputs
        self._J = (C.c_void_p * nb)(*[j._h for j in jobs])
        self._S = (C.c_void_p * nb)(*[_stream(s).value for s in streams])
        self._A = (C.c_void_p * nb)(*[_ptr(a).value for a in arc_bufs])
        self._F = (C.c_void_p * nb)(*[_ptr(f).value for f in feas_bufs])
        self.nb, self.B, self.spl = nb, int(B), int(steps_per_launch)
        h = C.c_void_p()
        check(lib().sspp_steps_create_sspp(self._J, nb, self._S, self.B, self.spl, self._A, self._F,
                                           C.byref(h)), "steps create")
        self._h = h
        self._run = lib().sspp_steps_run
        self._free = lib().sspp_steps_free

    def enqueue(self, nsteps, first_id, step_stride, best=None):
        """best: None, an (nsteps, 4) int64 device tensor for the per-step argmin records, or
        that tensor's device address as an int (callers in a timed loop cache it)."""
        bp = best if (best is None or isinstance(best, int)) else best.data_ptr()
        rc = self._run(self._h, nsteps, first_id, step_stride, bp)
        if rc:
            check(rc, "steps enqueue")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._free(h)
            self._h = None


class CesPlanner:
    """tsp::Planner's CES iteration on the device (include/sspp/tsp_planner.h:72-145).

    One iteration = begin (reset() or keep the distribution; seed list [mean set, forwarded
    best, samples]) -> eval (k_tsp over the slots) -> update (elites, Distribution::update,
    best, adapt) — all asynchronous on `stream`.  With world > 1 every rank owns
    slots_per_rank consecutive slots: `step` evaluates this rank's slots, all-gathers the
    per-slot results (one RCCL all_gather of a packed f64 record per slot) and runs the same
    update on every rank, so all ranks hold the identical distribution afterwards.

    Arguments follow tsp::TaskSpacePlanner's constructor (include/sspp/tsp.h:12-33); the
    planner's Distribution::z_min is `stddev_initial` as in the reference.
    """

    def __init__(self, scene, stddev_initial=0.3, stddev_min=0.01, stddev_max=0.5,
                 stddev_increase_factor=1.5, stddev_decay_factor=0.95, elite_fraction=0.3,
                 sample_count=50, check_points=50, init_points=3, collision_weight=1.0,
                 z_min=0.0, limits_min=(-2.0,) * 4, limits_max=(2.0,) * 4, sigma_floor=0.0,
                 var_ema_beta=0.2, mean_lr=0.5, floor_margin=0.01, floor_penalty_scale=10.0,
                 seed=DEFAULT_SEED, world=1, rank=0, group=None):
        self.lo, self.hi = _f64(limits_min, 4), _f64(limits_max, 4)
        cfg = CesConfig(samples=int(sample_count), checks=int(check_points),
                        total_points=int(init_points), w_collision=float(collision_weight),
                        elite_fraction=float(elite_fraction), inc=float(stddev_increase_factor),
                        dec=float(stddev_decay_factor), sigma_floor=float(sigma_floor),
                        var_beta=float(var_ema_beta), mean_lr=float(mean_lr),
                        stddev_min=float(stddev_min), stddev_max=float(stddev_max),
                        z_min=float(z_min), dist_z_min=float(stddev_initial), sigma0=0.3,
                        lo=_dptr(self.lo), hi=_dptr(self.hi),
                        # Planner never forwards cfg.z_min/floor_* to its Evaluator
                        floor_z_min=0.0, floor_margin=0.01, floor_scale=10.0,
                        seed=int(seed) & (2 ** 64 - 1))
        self.cfg = cfg
        self.configured_floor = (float(z_min), float(floor_margin), float(floor_penalty_scale))
        h = C.c_void_p()
        check(lib().sspp_ces_create(scene.handle, C.byref(cfg), int(world), C.byref(h)), "ces create")
        self._h = h
        self.scene, self.world, self.rank, self.group = scene, int(world), int(rank), group
        inf = CesInfo()
        check(lib().sspp_ces_get_info(self._h, C.byref(inf)), "ces info")
        self.K, self.n_slots, self.spr = inf.n_vias, inf.n_slots, inf.slots_per_rank
        self.samples = int(sample_count)
        b = CesBuffers()
        check(lib().sspp_ces_get_buffers(self._h, C.byref(b)), "ces buffers")
        self._bufs = b

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.sspp_ces_free(self._h)
            self._h = None

    def set_option(self, key, value):
        """Explicit option (SSPP_OPT_CES_FUSED); every setting gives bit-identical iterations."""
        check(lib().sspp_ces_set_option(self._h, int(key), int(value)), "ces set_option")

    def begin(self, start, end, iterate, stream=None):
        self._se = (_f64(start, 4), _f64(end, 4))
        check(lib().sspp_ces_begin(self._h, _dptr(self._se[0]), _dptr(self._se[1]),
                                   int(bool(iterate)), _stream(stream)), "ces begin")

    def eval(self, rank=None, stream=None):
        check(lib().sspp_ces_eval(self._h, self.rank if rank is None else int(rank),
                                  _stream(stream)), "ces eval")

    def update(self, stream=None):
        check(lib().sspp_ces_update(self._h, _stream(stream)), "ces update")

    def step(self, start, end, iterate, stream=None):
        """One plan() iteration on this rank (collective over the group when world > 1)."""
        self.begin(start, end, iterate, stream)
        self.eval(stream=stream)
        if self.world > 1:
            self._exchange(stream)
        self.update(stream)

    def _exchange(self, stream=None):
        """All-gather every rank's slot records (one collective), then unpack them into this
        rank's planner so the update sees the whole candidate list.

        Pack, gather and unpack are all ordered on `stream`: the collective is issued with
        `stream` as torch's current stream (RCCL orders its work after the current stream's
        and makes the current stream wait for the result), so a planner driven on a
        non-default stream cannot gather before the pack or unpack before the gather."""
        torch = _torch()
        rec = 5 + 4 * self.K
        if getattr(self, "_xbuf", None) is None:
            dev = torch.device("cuda", torch.cuda.current_device())
            self._xbuf = (torch.empty(self.spr * rec, dtype=torch.float64, device=dev),
                          torch.empty(self.world * self.spr * rec, dtype=torch.float64, device=dev))
        local, full = self._xbuf
        with torch.cuda.stream(torch_stream(stream)):
            check(lib().sspp_ces_pack(self._h, self.rank, _ptr(local), _stream(stream)), "ces pack")
            all_gather_records(full, local, self.group)
            check(lib().sspp_ces_unpack(self._h, _ptr(full), _stream(stream)), "ces unpack")

    def plan(self, start, end, iterate=False, iterations=1, stream=None):
        """iterations x plan(start, end, iterate) without host synchronisation (world == 1)."""
        if self.world > 1:
            for t in range(int(iterations)):
                self.step(start, end, iterate or t > 0, stream)
            return
        s, e = _f64(start, 4), _f64(end, 4)
        check(lib().sspp_ces_plan(self._h, _dptr(s), _dptr(e), int(bool(iterate)),
                                  int(iterations), _stream(stream)), "ces plan")

    @staticmethod
    def plan_group(planners, starts, ends, iterate=False, iterations=1, stream=None):
        """iterations x plan(start_g, end_g, iterate) of every planner, as one chain of batched
        launches on `stream` (sspp_ces_plan_group: one k_tsp_group per iteration over every
        goal's slots).  Each planner's results equal its own plan(); single-rank planners that
        share the scene, vias, checks, bounds and CES configuration (others run one by one)."""
        pls = list(planners)
        G = len(pls)
        s = _f64(np.asarray(starts, dtype=np.float64).reshape(G, 4), 4 * G)
        e = _f64(np.asarray(ends, dtype=np.float64).reshape(G, 4), 4 * G)
        hs = (C.c_void_p * G)(*[p._h.value for p in pls])
        check(lib().sspp_ces_plan_group(C.cast(hs, C.c_void_p), G, _dptr(s), _dptr(e), int(bool(iterate)), int(iterations),
                                        _stream(stream)), "ces plan group")

    def read(self):
        """Synchronous copy of the last iteration: per-candidate results and the state."""
        st = CesState()
        n, K = self.samples + 2, self.K
        L, Cnf, Cwf, cost = (np.zeros(n) for _ in range(4))
        status = np.zeros(n, np.uint8)
        vias = np.zeros((n, K, 4))
        mean, sigma, lbest = np.zeros((K, 4)), np.zeros((K, 4)), np.zeros((K, 4))
        elites = np.zeros(max(1, n), np.int32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        check(lib().sspp_ces_read(self._h, C.byref(st), p(L), p(Cnf), p(Cwf), p(cost), p(status),
                                  p(vias), p(mean), p(sigma), p(lbest), p(elites)), "ces read")
        m = st.n_candidates
        return dict(n_fixed=st.n_fixed, n_candidates=m, n_success=st.n_success,
                    n_elite=st.n_elite, has_best=bool(st.has_best), best_slot=int(st.best_slot),
                    best_cost=st.best_cost, iteration=int(st.iteration), L=L[:m], C_nf=Cnf[:m],
                    C_wf=Cwf[:m], cost=cost[:m], status=status[:m], vias=vias[:m], mean=mean,
                    sigma=sigma, last_best=lbest, elites=elites[:st.n_elite].copy())

    def set_state(self, mean=None, sigma=None, last_best=None, has_best=-1):
        """Overwrite the device distribution (test / warm-start hook; synchronous)."""
        keep = [None if a is None else _f64(a, 4 * self.K) for a in (mean, sigma, last_best)]
        ptrs = [None if a is None else a.ctypes.data_as(C.c_void_p) for a in keep]
        check(lib().sspp_ces_set_state(self._h, *ptrs, int(has_best)), "ces set_state")


def torch_stream(stream):
    """A torch stream object for `stream` (None = current, raw hipStream_t int = external)."""
    torch = _torch()
    if stream is None:
        return torch.cuda.current_stream()
    if isinstance(stream, int):
        return torch.cuda.ExternalStream(stream)
    return stream


def all_gather_records(out, local, group=None):
    """all_gather_into_tensor of device records on torch's current stream.  RCCL ("nccl")
    gathers device memory directly over xGMI; a gloo group (the CPU tests' backend) is staged
    through host memory, in the same stream order."""
    import torch.distributed as dist
    torch = _torch()
    if dist.get_backend(group) == "gloo":
        host = local.cpu()  # waits for the current stream's work on `local`
        parts = [torch.empty_like(host) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, host, group=group)
        out.copy_(torch.stack(parts).view(out.shape))
        return
    dist.all_gather_into_tensor(out, local, group=group)


def reduce_best_steps(parts, out, stream=None):
    """parts: (R, G, 4) int64 device tensor of per-rank step records -> out (G, 4)."""
    R, G = parts.shape[0], parts.shape[1]
    check(lib().sspp_best_reduce_steps(_ptr(parts), int(R), int(G), _ptr(out), _stream(stream)),
          "reduce_best_steps")


def device_count():
    n = C.c_int()
    rc = lib().sspp_device_count(C.byref(n))
    return n.value if rc == 0 else 0


__all__ = ["Model", "Scene", "SsppJob", "TspJob", "CesPlanner", "SsppSteps", "reduce_best_steps", "all_gather_records",
           "torch_stream", "interpolate", "spline_eval", "best_tensor", "check_records",
           "decode_best", "reduce_best", "reduce_best_device", "device_count", "DEFAULT_SEED",
           "SAMPLER_FP64", "SAMPLER_FP32", "math"]

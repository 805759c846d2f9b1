"""ctypes binding of include/sspp_hip.h (libsspp_hip.so, built in-tree by `make`).

Fails loudly: if the HIP library is missing or does not export a declared symbol, importing
the product raises — there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB_PATH = os.path.join(_HERE, "lib", "libsspp_hip.so")
# SSPP_LIB_PATH: a profiling variant (tools/build_variant.sh); never set on the product path
LIB_PATH = os.environ.get("SSPP_LIB_PATH") or PRODUCT_LIB_PATH
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "sspp_hip.h")

SSPP_OK = 0
SSPP_E_INCOMPLETE = -7  # a result record reports lost work (sspp_best::reserved != 0)
MODE_QPOS = 0
MODE_BODY = 1


class SsppError(RuntimeError):
    pass


class ModelView(C.Structure):
    _fields_ = [
        ("nbody", C.c_int), ("body_parent", C.POINTER(C.c_int32)),
        ("body_jnt_type", C.POINTER(C.c_int32)), ("body_qpos_adr", C.POINTER(C.c_int32)),
        ("body_pos", C.POINTER(C.c_double)), ("body_quat", C.POINTER(C.c_double)),
        ("ngeom", C.c_int), ("geom_type", C.POINTER(C.c_int32)),
        ("geom_body", C.POINTER(C.c_int32)), ("geom_contype", C.POINTER(C.c_int32)),
        ("geom_conaffinity", C.POINTER(C.c_int32)), ("geom_size", C.POINTER(C.c_double)),
        ("geom_pos", C.POINTER(C.c_double)), ("geom_quat", C.POINTER(C.c_double)),
        ("geom_margin", C.POINTER(C.c_double)), ("nexclude", C.c_int),
        ("exclude", C.POINTER(C.c_int32)), ("nq", C.c_int), ("qpos0", C.POINTER(C.c_double)),
    ]


class Best(C.Structure):
    _fields_ = [("cost", C.c_double), ("index", C.c_int64), ("count", C.c_int64),
                ("reserved", C.c_int64)]


class SceneInfo(C.Structure):
    _fields_ = [("n_moving_geoms", C.c_int), ("n_static_geoms", C.c_int), ("n_pairs", C.c_int),
                ("n_static_pairs", C.c_int), ("static_contacts", C.c_int),
                ("n_movers", C.c_int), ("static_cost", C.c_double)]


class SsppArgs(C.Structure):
    _fields_ = [("knots", C.POINTER(C.c_double)), ("degree", C.c_int),
                ("init_ctrl", C.POINTER(C.c_double)), ("n_ctrl", C.c_int), ("dof", C.c_int),
                ("sigma", C.c_double), ("limits", C.POINTER(C.c_double)),
                ("check_points", C.c_int), ("seed", C.c_uint64), ("arc_all", C.c_int),
                ("sampler", C.c_int)]


class TspArgs(C.Structure):
    _fields_ = [("start", C.POINTER(C.c_double)), ("end", C.POINTER(C.c_double)),
                ("n_vias", C.c_int), ("check_points", C.c_int), ("w_collision", C.c_double),
                ("mean", C.POINTER(C.c_double)), ("sigma", C.POINTER(C.c_double)),
                ("lo", C.POINTER(C.c_double)), ("hi", C.POINTER(C.c_double)),
                ("z_min", C.c_double), ("seed", C.c_uint64), ("floor_z_min", C.c_double),
                ("floor_margin", C.c_double), ("floor_scale", C.c_double)]


class CesConfig(C.Structure):
    _fields_ = [("samples", C.c_int), ("checks", C.c_int), ("total_points", C.c_int),
                ("w_collision", C.c_double), ("elite_fraction", C.c_double), ("inc", C.c_double),
                ("dec", C.c_double), ("sigma_floor", C.c_double), ("var_beta", C.c_double),
                ("mean_lr", C.c_double), ("stddev_min", C.c_double), ("stddev_max", C.c_double),
                ("z_min", C.c_double), ("dist_z_min", C.c_double), ("sigma0", C.c_double),
                ("lo", C.POINTER(C.c_double)), ("hi", C.POINTER(C.c_double)),
                ("floor_z_min", C.c_double), ("floor_margin", C.c_double),
                ("floor_scale", C.c_double), ("seed", C.c_uint64)]


class CesInfo(C.Structure):
    _fields_ = [("n_vias", C.c_int), ("n_slots", C.c_int), ("slots_per_rank", C.c_int),
                ("world", C.c_int), ("elite_capacity", C.c_int), ("iteration", C.c_int64)]


class CesState(C.Structure):
    _fields_ = [("n_fixed", C.c_int), ("n_candidates", C.c_int), ("n_success", C.c_int),
                ("n_elite", C.c_int), ("has_best", C.c_int), ("best_slot", C.c_int64),
                ("best_cost", C.c_double), ("iteration", C.c_int64)]


class CesBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("L", "C_nf", "C_wf", "cost", "status", "vias", "mean",
                                          "sigma", "last_best", "elites")]


_vp, _i64, _d, _i = C.c_void_p, C.c_int64, C.POINTER(C.c_double), C.c_int

SIGNATURES = {
    "sspp_last_error": (C.c_char_p, []),
    "sspp_version": (C.c_int, []),
    "sspp_build_id": (C.c_char_p, []),
    "sspp_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "sspp_model_load_mjcf": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "sspp_model_view_get": (C.c_int, [_vp, C.POINTER(ModelView)]),
    "sspp_model_body_id": (C.c_int, [_vp, C.c_char_p]),
    "sspp_model_geom_id": (C.c_int, [_vp, C.c_char_p]),
    "sspp_model_body_point": (C.c_int, [_vp, C.c_char_p, _d]),
    "sspp_model_free": (None, [_vp]),
    "sspp_scene_create": (C.c_int, [_vp, _i, _i, _i, C.POINTER(_vp)]),
    "sspp_scene_get_info": (C.c_int, [_vp, C.POINTER(SceneInfo)]),
    "sspp_scene_free": (None, [_vp]),
    "sspp_interpolate": (C.c_int, [_d, _i, _i, _i, _d, _d, _d]),
    "sspp_spline_eval": (C.c_int, [_d, _i, _i, _d, _i, C.c_double, _d]),
    "sspp_job_create_sspp": (C.c_int, [_vp, C.POINTER(SsppArgs), _i64, C.POINTER(_vp)]),
    "sspp_job_sample_score": (C.c_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp]),
    "sspp_job_score_ctrl": (C.c_int, [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "sspp_job_create_tsp": (C.c_int, [_vp, C.POINTER(TspArgs), _i64, C.POINTER(_vp)]),
    "sspp_job_tsp_sample_score": (C.c_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _vp]),
    "sspp_job_tsp_score_vias": (C.c_int, [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp]),
    "sspp_job_info": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                C.POINTER(C.c_size_t)]),
    "sspp_job_free": (None, [_vp]),
    "sspp_best_reduce": (C.c_int, [C.POINTER(Best), _i, C.POINTER(Best)]),
    "sspp_best_check": (C.c_int, [C.POINTER(Best), _i]),
    "sspp_best_reduce_device": (C.c_int, [_vp, _i, _vp, _vp]),
    "sspp_best_reduce_steps": (C.c_int, [_vp, _i, _i, _vp, _vp]),
    "sspp_steps_enqueue_sspp": (C.c_int, [C.POINTER(_vp), _i, C.POINTER(_vp), _i64, _i, _i,
                                          _i64, _i64, C.POINTER(_vp), C.POINTER(_vp), _vp]),
    "sspp_steps_create_sspp": (C.c_int, [C.POINTER(_vp), _i, C.POINTER(_vp), _i64, _i, C.POINTER(_vp),
                                         C.POINTER(_vp), C.POINTER(_vp)]),
    "sspp_steps_run": (C.c_int, [_vp, _i, _i64, _i64, _vp]),
    "sspp_steps_free": (None, [_vp]),
    "sspp_plan_sspp": (C.c_int, [_vp, _i, _d, _d, C.c_double, _d, _i, _i, _i, C.c_uint64, _d, _d,
                                 C.POINTER(C.c_uint8), _d, C.POINTER(Best)]),
    "sspp_score_ctrl_host": (C.c_int, [_vp, _d, _i, _d, _i64, _i, _i, _i, _d,
                                       C.POINTER(C.c_uint8), C.POINTER(Best)]),
    "sspp_sample_ctrl_host": (C.c_int, [_d, _i, _d, _i, _i, C.c_double, _d, C.c_uint64, _i64,
                                        _i64, _d]),
    "sspp_job_update_sspp": (C.c_int, [_vp, _d, C.c_double, _d, C.c_uint64, _vp]),
    "sspp_planner_create": (C.c_int, [_vp, _i, C.POINTER(_vp)]),
    "sspp_planner_plan": (C.c_int, [_vp, _d, _d, C.c_double, _d, _i, _i, _i, C.c_uint64, _i64, _d,
                                    C.POINTER(_i64), C.POINTER(_i64), _d, _d, C.POINTER(Best)]),
    "sspp_planner_score": (C.c_int, [_vp, _d, _i, _d, _i64, _i, _i, _i, _d, C.POINTER(C.c_uint8),
                                     C.POINTER(Best)]),
    "sspp_planner_free": (None, [_vp]),
    "sspp_planner_get_option": (C.c_int, [_vp, _i, C.POINTER(_i64)]),
    "sspp_ces_create": (C.c_int, [_vp, C.POINTER(CesConfig), _i, C.POINTER(_vp)]),
    "sspp_ces_get_info": (C.c_int, [_vp, C.POINTER(CesInfo)]),
    "sspp_ces_begin": (C.c_int, [_vp, _d, _d, _i, _vp]),
    "sspp_ces_eval": (C.c_int, [_vp, _i, _vp]),
    "sspp_ces_update": (C.c_int, [_vp, _vp]),
    "sspp_ces_plan": (C.c_int, [_vp, _d, _d, _i, _i, _vp]),
    "sspp_ces_plan_group": (C.c_int, [_vp, _i, _d, _d, _i, _i, _vp]),
    "sspp_ces_get_buffers": (C.c_int, [_vp, C.POINTER(CesBuffers)]),
    "sspp_ces_read": (C.c_int, [_vp, C.POINTER(CesState), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp]),
    "sspp_ces_set_state": (C.c_int, [_vp, _vp, _vp, _vp, _i]),
    "sspp_ces_pack": (C.c_int, [_vp, _i, _vp, _vp]),
    "sspp_ces_unpack": (C.c_int, [_vp, _vp, _vp]),
    "sspp_ces_free": (None, [_vp]),
    "sspp_job_set_option": (C.c_int, [_vp, _i, _i64]),
    "sspp_job_get_option": (C.c_int, [_vp, _i, C.POINTER(_i64)]),
    "sspp_ces_set_option": (C.c_int, [_vp, _i, _i64]),
}

# job options (include/sspp_hip.h SSPP_OPT_*)
OPT_SHAPE_NT, OPT_SHAPE_G1, OPT_ORDER, OPT_TSP_FORM, OPT_TSP_GENERIC = 1, 2, 3, 4, 5
OPT_SAMPLER, OPT_LAST_NT, OPT_LAST_G1, OPT_WP_ORDER, OPT_PREPASS_US, OPT_NPAIRS = 6, 7, 8, 9, 10, 11
OPT_CYLBOX, OPT_F32, OPT_LAST_F32, OPT_CREATE_US, OPT_PREPASS_STATE = 12, 13, 14, 15, 16
OPT_SPLIT, OPT_LAST_SPLIT, OPT_TSP_REP = 17, 18, 19
OPT_SPLIT_LINGER_US, OPT_SPLIT_DROP, OPT_SPLIT_HANDOFFS, OPT_SPLIT_LOST = 20, 21, 22, 23
OPT_CES_FUSED = 101


def declared_symbols(header=HEADER_PATH):
    """Function names declared in include/sspp_hip.h."""
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sspp_[a-z_0-9]+)\s*\(", txt)))


_lib = None
build_warning = None  # set when the product library's revision differs from the tree's


def check_revision(L, path, variant):
    """Compare the library's source stamp (sspp_build_id) with the tree's (sspp_amd/_stamp.py).
    A profiling variant from other sources is refused (its numbers would describe another
    revision, and a missing export would surface later as an AttributeError); a product library
    that differs is reported through `build_warning` (warnings.warn)."""
    from ._stamp import source_hash
    tree = source_hash()
    f = getattr(L, "sspp_build_id", None)
    built = None
    if f is not None:
        f.restype, f.argtypes = C.c_char_p, []
        built = (f() or b"").decode(errors="replace")
    if tree is None or built == tree:
        return None
    what = ("built from sources %s" % built) if built else "no source stamp (sspp_build_id)"
    msg = "%s: %s, but the tree's sources are %s" % (path, what, tree)
    if variant:
        raise SsppError("stale variant library " + msg +
                        " (rebuild it: bash tools/build_variant.sh NAME FLAGS)")
    import warnings
    warnings.warn("libsspp_hip.so does not match its sources: " + msg + " (run `make`)", RuntimeWarning)
    return msg


def lib():
    global _lib, build_warning
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SsppError("HIP library not built: %s (run `make` or __graft_entry__.build())"
                            % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        build_warning = check_revision(L, LIB_PATH, os.path.abspath(LIB_PATH) != PRODUCT_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)  # AttributeError -> missing export: fail loudly
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error():
    return lib().sspp_last_error().decode(errors="replace")


def check(rc, what=""):
    if rc < 0:
        msg = last_error()
        raise SsppError("%s failed (%d): %s" % (what, rc, msg))
    return rc

"""sspp_amd — MI355X-native candidate scoring for the sampled-spline path planner.

Product layout:
  csrc/              HIP kernels (gfx950) + C ABI (include/sspp_hip.h) + MJCF loader
  lib/               built libsspp_hip.so (in-tree)
  runtime.py         Model / Scene / SsppJob / TspJob over the C ABI
  BSplines.py, CubicPath.py   reference operator API (sspp/BSplines.py, sspp/CubicPath.py)
  scenes/            collision-only MJCF scenes derived from the reference's mjcf/
"""
import os

SCENE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")

from ._lib import (OPT_CES_FUSED, OPT_F32, OPT_ORDER, OPT_SPLIT, OPT_SHAPE_G1, OPT_SHAPE_NT, OPT_TSP_FORM,  # noqa: E402
                   OPT_TSP_GENERIC, OPT_TSP_REP, SsppError)
from .runtime import (DEFAULT_SEED, SAMPLER_FP32, SAMPLER_FP64, CesPlanner, Model, Scene, SsppJob, SsppSteps, TspJob,  # noqa: E402
                      all_gather_records, best_tensor, check_records, decode_best, device_count, interpolate,
                      reduce_best, reduce_best_device, reduce_best_steps, spline_eval, torch_stream)

__all__ = ["SsppError", "Model", "Scene", "SsppJob", "TspJob", "CesPlanner", "interpolate", "spline_eval",
           "best_tensor", "check_records", "decode_best", "reduce_best", "reduce_best_device", "reduce_best_steps",
           "SsppSteps", "all_gather_records", "torch_stream", "device_count", "DEFAULT_SEED", "SCENE_DIR",
           "SAMPLER_FP64", "SAMPLER_FP32", "OPT_SHAPE_NT", "OPT_SHAPE_G1", "OPT_ORDER", "OPT_TSP_FORM",
           "OPT_TSP_GENERIC", "OPT_TSP_REP", "OPT_CES_FUSED", "OPT_F32", "OPT_SPLIT"]

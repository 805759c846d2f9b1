"""Pair work of the TaskSpacePlanner evaluation (point_collide), per waypoint lane: lane pair
iterations after the hull masks, pairs past the sphere tests, by type, and deep contacts.  Needs
a -DSSPP_TSP_STATS variant via SSPP_LIB_PATH (bash tools/build_variant.sh tstats "-DSSPP_TSP_STATS").
    python tools/tsp_stats.py [stacking|multigoal]"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sspp_amd import _lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "stacking"
sys.argv = ["bench.py", "--config", cfg, "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
args = bench.parse()
device = torch.device("cuda", 0)
if cfg == "stacking":
    B, step, kernel_only, *_ = bench.setup_stacking(args, device)
    run = lambda: kernel_only(0)  # noqa: E731
else:
    B, step, kernel_only, *_ = bench.setup_multigoal(args, device, 1, 0)
    run = lambda: kernel_only(0)  # noqa: E731
f = _lib.lib().__getattr__("sspp_debug_tsp_stats")
buf = (C.c_ulonglong * 16)()
run()
torch.cuda.synchronize()
f(buf, 1)
run()
torch.cuda.synchronize()
f(buf, 1)
v = list(buf)
names = {0: "lane_pair_iters", 1: "near", 2: "near_box_box", 3: "near_cylinder", 4: "near_plane", 5: "deep"}
print(json.dumps({"config": cfg, "waypoint_lanes": v[6],
                  "per_waypoint_lane": {names[i]: v[i] / max(1, v[6]) for i in names}}, indent=1))

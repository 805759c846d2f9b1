"""Work statistics of k_sspp_c2f (needs a -DSSPP_C2F_STATS variant via SSPP_LIB_PATH):
    python tools/c2f_stats.py [NTxG1]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sspp_amd as S  # noqa: E402
from sspp_amd import _lib  # noqa: E402

model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
scene = S.Scene(model, 0, 7)
start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
u = np.array([i / 9 for i in range(10)])
knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
B = 4096
job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=B)
if len(sys.argv) > 1:  # a forced launch shape NTxG1 (default: the library's per-launch choice)
    job.set_shape(*(int(x) for x in sys.argv[1].lower().split("x")))
out = job.alloc(B)
f = _lib.lib().__getattr__("sspp_debug_c2f_stats")
buf = (C.c_ulonglong * 16)()
f(buf, 1)
for i in range(20):
    job.sample_score(i * B, B, out["arc"], out["feasible"], out["best"])
torch.cuda.synchronize()
f(buf, 1)
v = list(buf)
n = v[7]
names = {0: "p1_wave_pair_iters", 1: "p1_lane_pair_tests", 2: "near_lane_tests(all)", 4: "p2_wave_pair_iters",
         5: "p2_lane_pair_tests", 6: "p1_survivors", 7: "candidates", 9: "p1_wave_narrowphase_iters",
         10: "p2_wave_narrowphase_iters", 13: "f32_wave_pair_iters", 3: "f32_lanes_past_culls",
         11: "p1_f64_fallback_lanes", 12: "p2_f64_fallback_lanes"}
print(json.dumps({names[i]: (v[i] / n if i != 7 else n) for i in names}, indent=1))
print("per candidate; feasible:", float(out["feasible"].float().mean()))

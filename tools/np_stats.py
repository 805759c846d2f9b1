"""Narrowphase path counters (needs a -DSSPP_C2F_STATS variant via SSPP_LIB_PATH): how often the
cylinder-box test gets past the SAT axes (11), past the witnesses into the candidate search
(12), and how many box-box deep tests run (13) / find a deep contact (14)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import sspp_amd as S  # noqa: E402
from sspp_amd import _lib  # noqa: E402

f = _lib.lib().__getattr__("sspp_debug_c2f_stats")
buf = (C.c_ulonglong * 16)()
model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
body = model.body_id("gripper_collision_with_block/")
scene = S.Scene(model, 1, body)
f(buf, 1)
for g, (st, en) in enumerate(bench.MULTIGOAL):
    pl = S.CesPlanner(scene, sample_count=4096, check_points=128, init_points=3,
                      limits_min=bench.MG_LO, limits_max=bench.MG_HI, seed=S.DEFAULT_SEED + g)
    pl.plan(st, en, iterate=False, iterations=3)
torch.cuda.synchronize()
f(buf, 1)
v = list(buf)
print(json.dumps({"cyl_box_tests": v[10], "past_sat": v[11], "to_candidate_search": v[12],
                  "box_box_deep_tests": v[13], "box_box_deep": v[14],
                  "candidates": 8 * 3 * 4098}, indent=1))
